// hbx_dist.hip -- the multi-GPU winner exchange of a candidate-sharded acquisition.
//
// Reference loop being sharded: bohb.py:133-152 (one get_config scores num_samples candidates and
// keeps the first index of the smallest max(1e-8, g)/max(l, 1e-8)).  Candidates are independent, so
// each GPU scores a contiguous shard with global indices (hbx_kde_acquire's index_base) and the only
// collective is here: one RCCL all-gather over xGMI of every rank's 48-byte result record, reduced on
// the device by (score, index) -- the smallest score, ties to the smallest global index, which is the
// reference's strict '<' over candidates in index order.  Ranks whose winners lie within each other's
// error bounds (AcqResult.rel) are flagged HBX_ACQ_NEAR_TIE for the host to re-resolve in the
// reference's arithmetic, as within one GPU.
#include <string.h>

#include <rccl/rccl.h>

#include "hbx_common.h"

#define HBX_RCCL(call)                                                                           \
  do {                                                                                           \
    ncclResult_t _r = (call);                                                                    \
    if (_r != ncclSuccess)                                                                       \
      return hbx_fail(HBX_ERR_HIP, "%s failed: %s (%s:%d)", #call, ncclGetErrorString(_r), __FILE__, \
                      __LINE__);                                                                 \
  } while (0)

// one thread: the global winner of nranks gathered records
__global__ void argmin_records_kernel(const AcqResult* __restrict__ all, int32_t nranks, AcqResult* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int best = -1;
  int32_t shortlist = 0;
  for (int r = 0; r < nranks; ++r) {
    const AcqResult a = all[r];
    shortlist += a.shortlist;
    if (a.index < 0 || !(a.score < INFINITY)) continue;
    if (best < 0 || a.score < all[best].score || (a.score == all[best].score && a.index < all[best].index)) best = r;
  }
  AcqResult o;
  if (best < 0) {
    o.index = -1;
    o.score = NAN;
    o.pdf_l = NAN;
    o.pdf_g = NAN;
    o.rel = 0.f;
    o.flags = 0;
    o.near = 0;
  } else {
    o = all[best];
    // ranks whose winner can still beat this one in the reference's arithmetic
    int near = 0, flags = 0;
    for (int r = 0; r < nranks; ++r) {
      const AcqResult a = all[r];
      if (a.index < 0 || !(a.score < INFINITY)) continue;
      if (r == best || a.score <= o.score * (1.0 + 1.0001 * ((double)a.rel + (double)o.rel))) {
        ++near;
        flags |= a.flags;
      }
    }
    o.flags = flags | (near > 1 ? HBX_ACQ_NEAR_TIE : 0);
    o.near = near;
  }
  o.shortlist = shortlist;
  *out = o;
}

extern "C" {

int64_t hbx_rccl_unique_id_bytes(void) { return (int64_t)sizeof(ncclUniqueId); }

int hbx_rccl_get_unique_id(void* id_out) {
  if (!id_out) return hbx_fail(HBX_ERR_ARG, "hbx_rccl_get_unique_id: null");
  ncclUniqueId id;
  HBX_RCCL(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return HBX_OK;
}

int hbx_rccl_comm_init(void** comm, int32_t nranks, const void* id, int32_t rank, int32_t device) {
  if (!comm || !id) return hbx_fail(HBX_ERR_ARG, "hbx_rccl_comm_init: null");
  if (nranks < 1 || rank < 0 || rank >= nranks) return hbx_fail(HBX_ERR_ARG, "rank %d of %d", rank, nranks);
  HBX_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c;
  HBX_RCCL(ncclCommInitRank(&c, nranks, uid, rank));
  *comm = (void*)c;
  return HBX_OK;
}

// the communicator's rank count as RCCL itself reports it (the bench line's world size)
int hbx_rccl_comm_count(void* comm, int32_t* count) {
  if (!comm || !count) return hbx_fail(HBX_ERR_ARG, "hbx_rccl_comm_count: null");
  int c = 0;
  HBX_RCCL(ncclCommCount((ncclComm_t)comm, &c));
  *count = c;
  return HBX_OK;
}

int hbx_rccl_comm_destroy(void* comm) {
  if (comm) HBX_RCCL(ncclCommDestroy((ncclComm_t)comm));
  return HBX_OK;
}

int64_t hbx_argmax_gather_bytes(int32_t nranks) { return (int64_t)nranks * (int64_t)sizeof(AcqResult); }

// local: this rank's result record (device, e.g. hbx_kde_result_ptr of its acquisition workspace);
// gather: device scratch of hbx_argmax_gather_bytes(nranks) (every rank's record after the call);
// out: device record of the global winner (index global, HBX_ACQ_NEAR_TIE when ranks' winners lie
// within each other's bounds).  One ncclAllGather on `stream`, then one reduction kernel.
int hbx_argmax_allreduce(const void* local, void* gather, void* out, int32_t nranks, void* rccl_comm, void* stream) {
  if (!local || !gather || !out || !rccl_comm) return hbx_fail(HBX_ERR_ARG, "hbx_argmax_allreduce: null");
  if (nranks < 1) return hbx_fail(HBX_ERR_ARG, "hbx_argmax_allreduce: nranks=%d", nranks);
  hipStream_t s = (hipStream_t)stream;
  HBX_RCCL(ncclAllGather(local, gather, sizeof(AcqResult), ncclUint8, (ncclComm_t)rccl_comm, s));
  hipLaunchKernelGGL(argmin_records_kernel, dim3(1), dim3(64), 0, s, (const AcqResult*)gather, nranks,
                     (AcqResult*)out);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// the same reduction over records gathered by another transport (e.g. torch.distributed / gloo):
// all: device AcqResult[nranks] -> out (device)
int hbx_argmax_records(const void* all, int32_t nranks, void* out, void* stream) {
  if (!all || !out || nranks < 1) return hbx_fail(HBX_ERR_ARG, "hbx_argmax_records: bad arguments");
  hipLaunchKernelGGL(argmin_records_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const AcqResult*)all,
                     nranks, (AcqResult*)out);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"
