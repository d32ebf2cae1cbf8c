// hbx_capi.cpp -- error plumbing and introspection entry points of libhbx.so (see include/hbx.h).
#include <cstddef>
#include <stdarg.h>
#include <stdio.h>

#include "hbx_common.h"

static thread_local char g_err[1024] = "";

int hbx_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

extern "C" {

const char* hbx_last_error(void) { return g_err; }

const char* hbx_version(void) { return "hbx 0.1.0 gfx950"; }

int64_t hbx_kde_param_bytes(void) { return (int64_t)HBX_PARAM_BYTES; }
int64_t hbx_kde_param_bw_offset(void) { return (int64_t)offsetof(KdeParams, bw); }

int64_t hbx_kde_est_bytes(void) { return (int64_t)sizeof(KdeEst); }

int64_t hbx_acq_result_bytes(void) { return (int64_t)sizeof(AcqResult); }

int32_t hbx_max_dims(void) { return HBX_MAX_D; }

}  // extern "C"
