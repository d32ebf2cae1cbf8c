/* hbx.h -- C ABI of libhbx.so, the MI355X (gfx950) engine for HpBandSter's data-parallel hot path:
 * BOHB's KDE acquisition (good/bad product-kernel KDE fit, l(x)/g(x) scoring, argmin) and the
 * successive-halving promotion.
 *
 * Conventions
 *   - Every pointer marked "device" is a HIP device pointer (e.g. torch.Tensor.data_ptr() of a
 *     ROCm tensor); "host" pointers are ordinary CPU memory.  The library allocates nothing
 *     per call: callers own outputs, workspaces and scratch (sized by the *_bytes helpers).
 *   - `stream` is a hipStream_t (NULL = default stream).  Calls only enqueue work, except
 *     hbx_kde_prepare, which synchronises `stream` once to upload the model parameters.
 *   - Return value 0 on success, a negative HBX_ERR_* code otherwise; the message is available
 *     from hbx_last_error() (thread-local).  Calls are reentrant; nothing is cached globally.
 *
 * Reference interfaces replaced (paths relative to the HpBandSter snapshot):
 *   hbx_seg_argsort(_ex) + hbx_kde_fit <- bohb.py:220-246 (BOHB.new_result refit:
 *                                      np.argsort + sm.nonparametric.KDEMultivariate(..,'normal_reference'))
 *   hbx_kde_refit                   <- bohb.py:211-251 (the same refit plus both KDEs' preparation, one call)
 *   hbx_kde_refit_sync              <- bohb.py:211-251 (the same, the output block on the host when it returns)
 *   hbx_kde_prepare                 <- KDEMultivariate.__init__ model state (statsmodels 0.12.2
 *                                      kernel_density.py:101-115)
 *   hbx_kde_acquire                 <- bohb.py:124-169 (the num_samples loop: pdf of l and g per
 *                                      candidate, minimize_me, strict-'<' argmin)
 *   hbx_kde_logpdf                  <- KDEMultivariate.pdf (kernel_density.py:162-196), fp32 log domain
 *   hbx_kde_pdf_exact               <- KDEMultivariate.pdf, fp64, reference operation order
 *   hbx_sh_promote(_ex)             <- HB_iteration.py:149-190 (SuccessiveHalving.process_results ranks)
 *   hbx_argmax_allreduce            <- bohb.py:150-152 'if val < best' across candidate shards on many GPUs
 *                                      (the reference has no multi-GPU path)
 */
#ifndef HBX_H_
#define HBX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBX_OK 0
#define HBX_ERR_ARG (-1)
#define HBX_ERR_HIP (-2)
#define HBX_ERR_UNSUPPORTED (-3)

/* ---- introspection ---------------------------------------------------------------------- */
const char* hbx_last_error(void);
const char* hbx_version(void);
int64_t hbx_kde_param_bytes(void);     /* bytes of one prepared KDE parameter block (device) */
int64_t hbx_kde_param_bw_offset(void); /* byte offset of the KDE's fp64 bandwidths bw[D] in that block */
int64_t hbx_kde_est_bytes(void);       /* bytes per candidate of hbx_kde_logpdf output */
int64_t hbx_acq_result_bytes(void);    /* bytes of the acquisition result record */
int32_t hbx_max_dims(void);            /* largest D accepted */

/* ---- KDE refit (BOHB.new_result) --------------------------------------------------------- */
int64_t hbx_sort_scratch_bytes(int64_t N);

/* Stable argsort of every segment's fp64 losses (np.argsort order: -inf < finite < +inf < NaN,
 * ties by position).  loss: device f64[N]; seg_off: device i64[B+1]; max_seg: host bound on the
 * longest segment; order: device i64[N], positions local to each segment. */
int hbx_seg_argsort(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                    int64_t* order, void* scratch, int64_t scratch_bytes, void* stream);

/* Tie order of the sorts (argsort split and promotion ranks).
 *   HBX_ORDER_NUMPY: numpy 1.26.4's default np.argsort on an AVX-512 host -- the order the reference's
 *     np.argsort(losses) (bohb.py:229) and np.argsort(np.argsort(losses)) (HB_iteration.py:180,240) give
 *     tied losses (crashed +inf runs, quantised losses): the vendored x86-simd-sort avx512_argsort
 *     <double> restated on the device (hpbandster_amd/csrc/hbx_npsort.h; oracle/np_argsort.py pinned
 *     by numpy's own outputs).  Segments without ties cost one check pass over the sorted order.
 *   HBX_ORDER_STABLE: ties by position. */
#define HBX_ORDER_NUMPY 0
#define HBX_ORDER_STABLE 1

/* hbx_seg_argsort with the tie order chosen (hbx_seg_argsort itself = HBX_ORDER_STABLE); scratch:
 * hbx_sort_scratch_bytes(N). */
int hbx_seg_argsort_ex(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                       int64_t* order, void* scratch, int64_t scratch_bytes, int32_t order_mode, void* stream);

/* Normal-reference bandwidths and observed level counts of the good (head n_good of the argsort)
 * and bad (tail n_bad) rows of every segment, bit-exact with numpy's np.std.
 * X: device f64[N][D]; order: from hbx_seg_argsort; n_good/n_bad: device i64[B] (0 = skip);
 * fac_good/fac_bad: device f64[B] = n**(-1/(4+D)) computed on the host with pow();
 * vartype: device i32[D] (0 = continuous, 1 = categorical).
 * Outputs: bw_* device f64[B][D]; nlev_* device i32[B][D] (-1 = categorical code not an
 * integer in [0, 1024)). */
int hbx_kde_fit(const double* X, int32_t D, const int64_t* seg_off, int64_t B, const int64_t* order,
                const int64_t* n_good, const int64_t* n_bad, const double* fac_good, const double* fac_bad,
                const int32_t* vartype, double* bw_good, double* bw_bad, int32_t* nlev_good, int32_t* nlev_bad,
                void* stream);

/* One-call refit of one budget's KDE pair (bohb.py:211-251: append the new observation(s), np.argsort
 * of the losses, good = head n_good / bad = tail n_bad rows, KDEMultivariate(.., 'normal_reference') for
 * both), enqueued on `stream` without host synchronisation; the caller reads `out` back once.
 *   X / loss: device f64[cap][D] / f64[cap] holding the budget's rows 0..n-1 after the call: rows
 *     n-n_new .. n-1 are copied in from `staged` (device f64[n_new*D + n_new]: rows, then losses;
 *     n_new = 0: X / loss are complete already).
 *   vartype: host i32[D] (0 = continuous, 1 = categorical); n_good / n_bad (bohb.py:224-225, clipped to
 *     n) and fac_* = n_good**(-1/(4+D)) / n_bad**(...) from the host's pow().
 *   params_* / table_*: as hbx_kde_prepare (tables of hbx_kde_table_floats(n_good|n_bad, ...) floats).
 *   out: device, hbx_kde_refit_out_bytes(n, D) bytes = order i64[n] | bw_good f64[D] | bw_bad f64[D] |
 *     nlev_good i32[D] | nlev_bad i32[D] | info_good i32[8] | info_bad i32[8] (info as hbx_kde_prepare);
 *     the KDEs' rows are order[0..n_good) and order[n-n_bad..n) -- keep `out` alive with the model.
 *     The argsort is numpy's (HBX_ORDER_NUMPY): tied losses give the reference's rows, in its order.
 *   scratch: device, hbx_kde_refit_scratch_bytes(n, D) bytes. */
int64_t hbx_kde_refit_out_bytes(int64_t n, int32_t D);
int64_t hbx_kde_refit_scratch_bytes(int64_t n, int32_t D);
int hbx_kde_refit(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype, const double* staged,
                  int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good, double fac_bad, void* params_good,
                  float* table_good, int64_t table_good_floats, void* params_bad, float* table_bad,
                  int64_t table_bad_floats, void* out, void* scratch, int64_t scratch_bytes, void* stream);
/* hbx_kde_refit with `staged_host` in HOST memory (rows, then losses: n_new*(D+1) doubles; up to 256 staged
 * doubles of a budget of at most 1024 rows ride in the kernel arguments of the refit's first launch, no
 * host-to-device copy; more go through `scratch`), synchronous: when the call returns, `out_host` (host memory,
 * hbx_kde_refit_out_bytes) holds the output block.  The preparation's launches publish it to a device-mapped
 * host buffer, every 32-bit word as an 8-byte word flagged with the call's sequence number, and the call spins
 * until every word carries it (no copy launch, no blocking stream synchronisation).  The prepared models are
 * complete for work enqueued on `stream` afterwards; work on ANOTHER stream must first be ordered after the
 * refit (hbx_stream_order(other, stream)).  The drop-in's ObservationStore.refit calls this one
 * (bohb.py:211-251, one new_result per call). */
int hbx_kde_refit_sync(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype,
                       const double* staged_host, int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good,
                       double fac_bad, void* params_good, float* table_good, int64_t table_good_floats,
                       void* params_bad, float* table_bad, int64_t table_bad_floats, void* out, void* scratch,
                       int64_t scratch_bytes, void* stream, void* out_host);
/* Order stream `waiter` after all work enqueued on `signaller` so far (event record + stream wait, no host
 * wait): a model refit / prepared on one stream, used from another. */
int hbx_stream_order(void* waiter, void* signaller);

/* ---- KDE model preparation ----------------------------------------------------------------- */
/* Template bucket of the scoring kernel for dc continuous / du categorical dims
 * (stride = floats per 64-observation table chunk). */
int hbx_kde_bucket(int32_t dc, int32_t du, int32_t* dc_pad, int32_t* du_pad, int32_t* stride);
/* floats of the observation table of an n-row KDE in bucket (dc_pad, du_pad) */
int64_t hbx_kde_table_floats(int32_t n, int32_t dc_pad, int32_t du_pad);

/* Build one KDE for scoring.  X: device f64[*][D]; rows: device i64[n] (this KDE's rows, in
 * the reference's order); vartype/bw/nlev: host arrays of length D.  params: device buffer of
 * hbx_kde_param_bytes(); table: device f32[hbx_kde_table_floats(n, dc_pad, du_pad)].  info: host i32[8] =
 * {variant, nan_all, unsupported, dc, du, nconst, dc_pad, du_pad}; variant = has_neg | kc << 1 selects
 * the scoring kernel (kc = 0: categorical matching on the VALU; kc >= 1: categorical one-hot product
 * on the f16 matrix cores with kc K-steps) and is passed back to hbx_kde_logpdf / hbx_kde_acquire. */
int hbx_kde_prepare(const double* X, int32_t D, const int64_t* rows, int32_t n, const int32_t* vartype,
                    const double* bw, const int32_t* nlev, void* params, float* table, int64_t table_floats,
                    int32_t* info, void* stream);

/* ---- scoring ------------------------------------------------------------------------------- */
/* fp32 log-domain sums for Nc candidates (device f64[Nc][D]) against one prepared KDE;
 * est_out: device, Nc * hbx_kde_est_bytes() ({ln S+, ln S-, rel. bound, pad} per candidate). */
int hbx_kde_logpdf(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                   int32_t dc_pad, int32_t du_pad, int32_t variant, void* est_out, void* stream);

int64_t hbx_kde_workspace_bytes(int64_t Nc, int64_t nmax);

/* One acquisition: l = good KDE, g = bad KDE; selects the first index of the minimum of
 * max(1e-8, g)/max(l, 1e-8) over the candidates, exactly (fp64 re-score of every candidate whose
 * fp32 score interval reaches the minimum).  index_base is added to the reported index (GPU
 * sharding).  logl_out/logg_out: nullable device f32[Nc]: the fp32 ln pdf point estimates the
 * selection used (-inf for pdf <= 0, NaN for NaN).  Each lies within its own rigorous bound (what keeps
 * the selection exact), which is 1e-5 relative at D <= 32 away from outlying observations but NOT in
 * general (the fp32 expansion -|x'|^2 - |X'|^2 + 2 x'.X' cancels large terms next to outliers and beyond
 * D = 32); ln pdfs within the north-star 1e-5 everywhere come from hbx_kde_logpdf_rtol.  With both NULL
 * the scoring runs the fast instance (the
 * one-hot deltas' f16 lo parts moved into the bound: looser estimates, the same exact selection).  The
 * result record lives in the workspace: hbx_kde_result_ptr(workspace).
 * events: NULL or hipEvent_t[3] (see hbx_event_create). */
int hbx_kde_acquire(const double* cand, int64_t Nc, int32_t D, int64_t index_base,
                    const void* params_good, const float* table_good, const double* X_good,
                    const int64_t* rows_good, int32_t variant_good,
                    const void* params_bad, const float* table_bad, const double* X_bad,
                    const int64_t* rows_bad, int32_t variant_bad, int32_t dc_pad, int32_t du_pad,
                    int64_t nmax, float* logl_out, float* logg_out, void* workspace, int64_t ws_bytes,
                    void* events, void* stream);

/* The synchronous acquisition (bohb.py:124-169 returns the pick to get_config's caller) on a KDE pair whose
 * fixed arguments (D, params_good .. nmax) are bound once: the drop-in binds each model it fits
 * (bohb.py:248-251 replaces the pair on every refit), and a call passes only what changes -- about 2 us less
 * host time per acquisition than converting all of them.  The handle holds the pointers only: the caller keeps
 * the KDEs' device buffers alive while it is in use, and frees it with hbx_kde_pair_free.  NULL on bad
 * arguments (hbx_last_error).
 * hbx_kde_acquire_bound: hbx_kde_acquire (fast scoring instances, no ln-pdf outputs) whose final kernel also
 * stores the 48-byte record into this thread's device-mapped host buffer, every 32-bit word as an 8-byte word
 * tagged with the call's sequence number; the call spins until every word carries its tag (bounded, then it
 * synchronises `stream`) and copies the record to rec_out (host, 48 bytes;
 * it also stays in the workspace, hbx_kde_result_ptr).  err (nullable, device u8[Nc], the GPU sampler's
 * domain-error flags): HBX_ACQ_DOMAIN_ERR is set in the record when any flag is set.  row_out (nullable, host
 * f64[D]): the winning candidate's row.  Both come with the record from the same final kernel: one wait for
 * the whole pick.  events: NULL or hipEvent_t[3] (hbx_kde_acquire). */
void* hbx_kde_pair_bind(int32_t D, const void* params_good, const float* table_good, const double* X_good,
                        const int64_t* rows_good, int32_t variant_good, const void* params_bad,
                        const float* table_bad, const double* X_bad, const int64_t* rows_bad, int32_t variant_bad,
                        int32_t dc_pad, int32_t du_pad, int64_t nmax);
int hbx_kde_acquire_bound(const void* pair, const double* cand, int64_t Nc, int64_t index_base, void* workspace,
                          int64_t ws_bytes, const uint8_t* err, void* events, void* stream, void* rec_out,
                          double* row_out);
void hbx_kde_pair_free(void* pair);

/* Batched acquisition: B = ceil(Nc / seg) independent get_config calls against the same model in one
 * pass (replaces B sequential runs of the bohb.py:124-169 loop, as an SH stage issues
 * them back to back, HB_iteration.py:136-138).  Candidates [b*seg, min((b+1)*seg, Nc)) belong to call b;
 * results: device buffer of B * hbx_acq_result_bytes() records, record b = call b's exact argmin with
 * the index relative to its segment start (+ index_base), -1 when the segment has no finite score.
 * Workspace: hbx_kde_batch_workspace_bytes(Nc, seg, nmax). */
int64_t hbx_kde_batch_workspace_bytes(int64_t Nc, int64_t seg, int64_t nmax);
int hbx_kde_acquire_batch(const double* cand, int64_t Nc, int64_t seg, int32_t D, int64_t index_base,
                          const void* params_good, const float* table_good, const double* X_good,
                          const int64_t* rows_good, int32_t variant_good,
                          const void* params_bad, const float* table_bad, const double* X_bad,
                          const int64_t* rows_bad, int32_t variant_bad, int32_t dc_pad, int32_t du_pad,
                          int64_t nmax, float* logl_out, float* logg_out, void* results, void* workspace,
                          int64_t ws_bytes, void* stream);

/* Optional timing: `events` of hbx_kde_acquire is NULL or an array of three hipEvent_t recorded on
 * `stream` before the l scoring launch, between l and g, and after g -- or, when l and g are scored by
 * one pair launch (both KDEs on the same hmode kernel, HBX_SCORE_PAIR not 0), only [0] before and [1]
 * after it. */
int hbx_event_create(void** ev);
int hbx_event_destroy(void* ev);
int hbx_event_elapsed_ms(void* start, void* stop, float* ms);

/* Copy `bytes` of device memory (e.g. the result record) to host memory on `stream` and wait for it without
 * a blocking synchronisation: up to 4096 bytes go through the calling thread's device-mapped host buffer
 * (allocated on the thread's first call and kept for its lifetime, ~8.4 KB with hbx_kde_acquire_bound's
 * tagged region; when the thread ends it goes back to a process-wide pool for the next thread) with a
 * completion word the
 * call spins on; larger or unaligned copies poll the stream.  Replaces the caller's copy + synchronise
 * after hbx_kde_acquire (the reference's get_config returns the pick to its caller: bohb.py:166). */
int hbx_fetch(void* host_dst, const void* dev_src, int64_t bytes, void* stream);

/* Device-mapped host buffers this process has allocated (hbx_fetch / hbx_kde_acquire_bound's and the refits'):
 * bounded by the threads calling at once, not by the threads that ever called -- a thread's buffer is pooled
 * when the thread ends.  Diagnostic (tests). */
int64_t hbx_mapped_host_buffers(void);

/* Device address of the result record inside an acquisition workspace (48 bytes):
 *   {i64 index, f64 score, f32 rel, i32 flags, i32 shortlist, i32 near, f64 pdf_l, f64 pdf_g}
 * index: first index of the minimal exact score (-1: no finite score); rel: bound of
 * |score - the same score in numpy's arithmetic| / score; near: candidates whose scores lie within those
 * bounds of the winner's (itself included).  flags: HBX_ACQ_OVERFLOW (1: every candidate re-scored),
 * HBX_ACQ_NEAR_TIE (2: near > 1 -- the fp64 re-score here and numpy may order them differently, so the
 * near set (hbx_kde_ws_offsets) must be re-scored in the reference's own arithmetic to pick the
 * reference's index; the Python wrapper does this on the host and sets HBX_ACQ_RESOLVED, 4). */
#define HBX_ACQ_OVERFLOW 1
#define HBX_ACQ_NEAR_TIE 2
#define HBX_ACQ_RESOLVED 4
#define HBX_ACQ_DOMAIN_ERR 8  /* hbx_kde_acquire_bound with err: a candidate's draw hit a domain error */
void* hbx_kde_result_ptr(void* workspace);
/* Byte offsets of [shortlist count (i32), shortlist (i32 candidate indices), near list, exact l (f64),
 * exact g (f64)] inside the workspace of an acquisition over (Nc, seg, nmax) candidates (seg = Nc for
 * hbx_kde_acquire).  hbx_kde_acquire's near list holds the near set's candidate indices (record.near of
 * them); hbx_kde_acquire_batch's holds a 0/1 flag per shortlist entry. */
int hbx_kde_ws_offsets(int64_t Nc, int64_t seg, int64_t nmax, int64_t* out);

int64_t hbx_kde_pdf_scratch_bytes(int64_t nmax);

/* Exact fp64 pdf of one prepared KDE at Np points (device f64[Np][D]) -> out (device f64[Np]).  Same
 * float64 operations in the same order as statsmodels 0.12.2 on the pinned numpy 1.26.4 (its SVML exp
 * restated bit for bit, numpy's pairwise sums): bit-identical to the reference's KDEMultivariate.pdf.
 * Np = 0: nothing to do (pts / out may be NULL); likewise hbx_kde_logpdf_exact. */
int hbx_kde_pdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                      const int64_t* rows, int64_t n, double* out, void* scratch, int64_t scratch_bytes,
                      void* stream);
/* ln KDEMultivariate.pdf (SM:kernel_density.py:162-196) in fp64 log space: logsumexp over the
 * observations of the log kernel products (no fp64 underflow, ~1e-15 relative).  NaN for KDEs with
 * negative categorical factors or structural NaNs -- use hbx_kde_pdf_exact there.  out: device f64[Np]. */
int hbx_kde_logpdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                         const int64_t* rows, double* out, void* stream);

/* ln pdf of one prepared KDE at Nc candidates within rtol * max(1, |ln pdf|) of the reference's
 * KDEMultivariate.pdf (kernel_density.py:162-196) -- the north-star contract at every D: the fp32
 * estimate (hbx_kde_logpdf) wherever its rigorous per-candidate bound guarantees rtol, the fp64 log-space
 * evaluation (hbx_kde_logpdf_exact) for the rest -- candidates next to outlying observations, beyond
 * D = 32, exact-only KDEs -- and ln of the exact fp64 pdf for KDEs with negative categorical factors.
 * All on the device.  cand: device f64[Nc][D]; X / rows: the KDE's observations (as hbx_kde_pdf_exact);
 * out: device f64[Nc] (-inf: pdf 0; NaN where the reference's pdf is NaN or negative);
 * scratch: hbx_kde_logpdf_rtol_scratch_bytes(Nc) device bytes. */
int64_t hbx_kde_logpdf_rtol_scratch_bytes(int64_t Nc);
int hbx_kde_logpdf_rtol(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                        const double* X, const int64_t* rows, int32_t dc_pad, int32_t du_pad, int32_t variant,
                        double rtol, double* out, void* scratch, int64_t scratch_bytes, void* stream);

/* numpy 1.26.4's float64 exp (what the reference's np.exp computes on AVX512_SKX hosts), element-wise
 * on the device: the known-answer check of the exact re-score's exp.  x, y: device f64[n]. */
int hbx_np_exp(const double* x, int64_t n, double* y, void* stream);

/* ---- candidate sampler (bohb.py:133-147, on the GPU) --------------------------------------- */
/* Philox4x32-10 block function (host): out[4] = philox(counter[4], key[2]).  Exposed for the
 * known-answer tests of the generator the sampler uses. */
int hbx_philox4x32_10(const uint32_t* counter, const uint32_t* key, uint32_t* out);

/* Nc candidates around the good KDE's observations, BOHB's rule: datum = rows[U{0..n-1}], then per
 * dim truncnorm(-m/bw, (1-m)/bw, loc=m, scale=bw_factor*bw) (levels[d] == 0) or keep-with-prob-(1-bw)
 * / U{0..t-1} (levels[d] = t).  X: device f64[*][D]; rows: device i64[n] (the good KDE's rows);
 * bw: device f64[D]; levels: device i32[D].  Dims 2k, 2k+1 of candidate i use Philox counter
 * (counter_base + i, k, stream_id) under key = seed (32-bit words: the uniform, the categorical level
 * draw), so consecutive calls with advancing counter_base equal one call over the union; the truncnorm
 * inversion is fp32 on the smaller tail (distributional parity).  cands: device f64[Nc][D], 16-byte
 * aligned when D is even; datum: nullable device i64[Nc] (drawn row positions);
 * domain_err: nullable device u8[Nc], 1 where a continuous dim's bounds fail scipy's a < b check
 * (the reference's call raises and falls back to a random configuration). */
int hbx_kde_sample(const double* X, int32_t D, const int64_t* rows, int64_t n, const double* bw,
                   const int32_t* levels, const double* tab, double bw_factor, uint64_t seed, uint64_t counter_base,
                   uint32_t stream_id, int64_t Nc, double* cands, int64_t* datum, uint8_t* domain_err, void* stream);
/* Standard normal quantile Phi^-1 (device f64[n] -> device f64[n]) in fp64 (Wichura's AS 241,
 * scipy.special.ndtri semantics on (0, 1)). */
int hbx_norm_ppf(const double* p, int64_t n, double* z, void* stream);
/* Optional per-model table for hbx_kde_sample (`tab`, nullable): Phi at the standardised truncnorm
 * bounds of every (good row, continuous dim), device f64[hbx_kde_sample_table_bytes(n, D) / 8].  Same
 * draws with or without it; it saves two normcdf per draw when Nc >> n. */
int64_t hbx_kde_sample_table_bytes(int64_t n, int32_t D);
int hbx_kde_sample_table(const double* X, int32_t D, const int64_t* rows, int64_t n, const double* bw,
                         const int32_t* levels, double* tab, void* stream);

/* ---- cross-validation bandwidth objectives (KDEMultivariate bw='cv_ls' / 'cv_ml') ------------ */
/* Per-observation sums of the CV objectives at bandwidths bw (SM:kernel_density.py:126-160,246-332;
 * the reference's caller: kde.py:145-147):
 *   F[i] = sum_j prod_d kbar_d(X_j, X_i) / bwprod     (convolution kernels; imse's first term)
 *   L[i] = sum_{j != i} prod_d k_d(X_j, X_i) / bwprod (leave-one-out kernels)
 * imse = sum_i F[i] / n^2 - 2 sum_i L[i] / (n (n-1)); loo log-likelihood = -sum_i log L[i] (host sums,
 * in order).  X: device f64[n][D]; vartype: device i32[D] (0 = 'c', 1 = 'u'); bw: device f64[D];
 * lev/lev_off: device, per categorical dim d the ascending unique values of -X[:, d] in
 * lev[lev_off[d] .. lev_off[d+1]) (continuous dims: empty); loo_levels: device i32[n][D], the level
 * count of column d without row i; c4 = 1/sqrt(4 pi), c2 = 1/sqrt(2 pi), bwprod = prod of the
 * continuous bandwidths in dim order (host).  F or L may be NULL (not computed). */
int hbx_kde_cv_terms(const double* X, int64_t n, int32_t D, const int32_t* vartype, const double* bw,
                     const double* lev, const int32_t* lev_off, const int32_t* loo_levels, double c4, double c2,
                     double bwprod, double* F, double* L, void* stream);

/* ---- multi-GPU winner exchange (candidate sharding; bohb.py:133-152 sharded) ----- */
/* Each rank runs hbx_kde_acquire on its contiguous shard with index_base = its first global index; the
 * ranks' result records then meet in ONE RCCL all-gather over xGMI and are reduced on the device by
 * (score, global index): the smallest score, ties to the smallest index -- the reference's strict '<'
 * in index order.  Winners within each other's error bounds set HBX_ACQ_NEAR_TIE (record.near = ranks
 * involved) for a host re-resolution.  ("argmax" of l/g = argmin of the BOHB score g/l.)
 *   local: this rank's device result record (hbx_kde_result_ptr); gather: device scratch of
 *   hbx_argmax_gather_bytes(nranks) holding every rank's record afterwards; out: device record of the
 *   global winner; rccl_comm: an ncclComm_t (hbx_rccl_comm_init, or the caller's own). */
int64_t hbx_rccl_unique_id_bytes(void);
int hbx_rccl_get_unique_id(void* id_out);
int hbx_rccl_comm_init(void** comm, int32_t nranks, const void* id, int32_t rank, int32_t device);
/* the communicator's rank count as RCCL reports it (ncclCommCount) */
int hbx_rccl_comm_count(void* comm, int32_t* count);
int hbx_rccl_comm_destroy(void* comm);
int64_t hbx_argmax_gather_bytes(int32_t nranks);
int hbx_argmax_allreduce(const void* local, void* gather, void* out, int32_t nranks, void* rccl_comm, void* stream);
/* The same reduction over records gathered by another transport (device AcqResult[nranks] -> out). */
int hbx_argmax_records(const void* all, int32_t nranks, void* out, void* stream);

/* ---- successive-halving promotion -------------------------------------------------------- */
/* advance[i] = rank_i < k[b] among the finite losses of bracket b (non-finite = CRASHED, never
 * advance; ties ranked by position).  loss: device f64[N]; seg_off: device i64[B+1]; k: device f64[B];
 * order: device i64[N] (sorted positions per bracket, output) or NULL when only the mask is wanted --
 * brackets of <= 1024 configurations then take an O(n) selection of the k-th loss and need no
 * scratch (scratch may be NULL); advance: device u8[N]; n_advance: device i64[B], nullable.
 * scratch: hbx_sort_scratch_bytes(N) bytes when order is requested or a bracket exceeds 1024.
 * N = 0 (every bracket empty): loss, order and advance may be NULL; n_advance is zeroed. */
int hbx_sh_promote(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                   const double* k, int64_t* order, uint8_t* advance, int64_t* n_advance, void* scratch,
                   int64_t scratch_bytes, void* stream);

/* hbx_sh_promote with the tie order chosen (hbx_sh_promote itself = HBX_ORDER_STABLE).  HBX_ORDER_NUMPY:
 * the finite losses of a bracket are ranked in numpy's argsort order (HB_iteration.py:179-180 sees only
 * the REVIEW configurations); brackets whose tied losses straddle the k-th place (or, with `order`
 * requested, hold any tie) are re-ranked on the device.  scratch: hbx_sh_promote_scratch_bytes(...)
 * bytes (never NULL in HBX_ORDER_NUMPY). */
int64_t hbx_sh_promote_scratch_bytes(int64_t B, int64_t max_seg, int64_t N, int32_t order_requested,
                                     int32_t order_mode);
int hbx_sh_promote_ex(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                      const double* k, int64_t* order, uint8_t* advance, int64_t* n_advance, void* scratch,
                      int64_t scratch_bytes, int32_t order_mode, void* events, void* stream);
/*   events: NULL, or hipEvent_t[2] stamped at the start and end of the selection kernel (mask-only path). */

/* One bracket of n <= 1024 configurations (what SuccessiveHalving.process_results ranks per call,
 * HB_iteration.py:179-182): a one-wave selection launch, then (HBX_ORDER_NUMPY) a re-rank launch that works
 * only when tied losses straddle the k-th place.  loss f64[n] and advance u8[n] may be device pointers or
 * mapped host memory from hbx_host_alloc (no copies); k by value; scratch: device int32[4 n]
 * (HBX_ORDER_NUMPY), or NULL (HBX_ORDER_STABLE).  done (nullable, mapped host memory): set to `seq` once
 * every mask byte is visible to the host, so a caller may poll it instead of synchronising the stream. */
int hbx_sh_promote_one(const double* loss, int64_t n, double k, uint8_t* advance, void* scratch, int32_t order_mode,
                       int32_t* done, int32_t seq, void* stream);
/* The same ranking step as ONE host call (what the drop-in's advance_mask makes): losses (host f64[n]) are
 * copied into `pin` (hbx_host_alloc, >= n doubles), the selection runs with advance = `pout`
 * (hbx_host_alloc, >= n bytes), the host spins on `done` (mapped, after pout) until the kernel stores
 * `seq` (> 0; bounded: then the stream is synchronised) -- or -seq: a straddling tie, the re-rank is
 * launched and waited for the same way -- and the mask is copied into `mask` (host u8[n]).
 * losses == pin (filled by the caller) and mask == pout (read by the caller) skip those copies.
 * Replaces np.argsort(np.argsort(losses)) < k of HB_iteration.py:179-182 for one bracket. */
int hbx_sh_advance_mapped(const double* losses, int64_t n, double k, uint8_t* mask, double* pin, uint8_t* pout,
                          int32_t* done, int32_t seq, void* scratch, int32_t order_mode, void* stream);
/* hbx_sh_advance_mapped with its buffers in a state block (4 arguments: what a per-call FFI hop costs, the
 * drop-in's advance_mask pays on every bracket): state = int64[7] {pin, pout, done, scratch, order_mode,
 * seq, device}.  The caller has written the losses into pin; the mask is left in pout; seq is advanced by
 * the call (1 ... 2^31 - 2, wrapping).  The launch runs on `device` (the scratch's; the stream must be one
 * of its streams) whichever device is current on the calling thread, which is left as it was. */
int hbx_sh_advance_state(int64_t* state, int64_t n, double k, void* stream);
/* Pinned, device-mapped, coherent host memory (hipHostMalloc) and its release. */
int hbx_host_alloc(int64_t bytes, void** out);
int hbx_host_free(void* p);

/* ---- numpy's argsort on the host (hbx_npsort_host.cpp) ------------------------------------------------
 * hbx_np_argsort_host: np.argsort(x) of numpy 1.26.4 on an AVX-512 host (x86-simd-sort avx512_argsort<double>,
 *   std::sort with NaN last when a NaN is present), ties in its order; host x[n] -> host order[n].
 * hbx_sh_advance_host: one bracket's HB_iteration.py:180-182 on the host: advance[i] = argsort(argsort(loss))[i]
 *   < k, i.e. the first k positions of that argsort; host loss[n], advance u8[n], scratch i64[n].
 *   Replaces np.argsort(np.argsort(losses)) < num_configs[SH_iter] of SuccessiveHalving.process_results for
 *   one bracket whose tied losses straddle the k-th place (hbx_sh_promote_ex ranks batched brackets). */
int hbx_np_argsort_host(const double* x, int64_t n, int64_t* order);
int hbx_sh_advance_host(const double* loss, int64_t n, int64_t k, uint8_t* advance, int64_t* scratch);

/* ---- BOHB's candidate draws on the host (bohb.py:133-147), the reference's RNG stream -------------
 * Host code (hbx_draw.cpp), no device work.  `state` is the MT19937 state a legacy numpy RandomState
 * holds (uint32 key[624] followed by int pos: hbx_mt_state_bytes() bytes, e.g. the global generator's
 * bit_generator.ctypes.state_address, held under that generator's lock); the draws continue its stream
 * exactly as the reference's calls would.
 * hbx_mt_draw: n draws of random_sample() (kind 0) or randint(0, high) (kind 1) into out (self-checks).
 * hbx_bohb_draw: one get_config call's draws -- per candidate randint(0, n) for the datum (bohb.py:135),
 *   then per dim of data[idx] (host f64[n][D]): levels[d] == 0 (continuous): scipy truncnorm.rvs's domain
 *   check (a = -m/bw < b = (1-m)/bw, scale = bw_factor bw >= 0; on failure *stop = element, return 1, the
 *   state left as the reference's raise leaves it), loc returned when scale == 0, else ONE uniform into
 *   uni[e] with need_ppf[e] = 1 and vals[e] = m (the caller computes truncnorm._ppf(uni, a, b) * scale + m,
 *   the rest of rvs); levels[d] > 0: rand() < 1 - bw keeps m, else randint(levels[d]) (bohb.py:144-147).
 *   vals/uni: host f64[num_samples][D]; need_ppf: host u8[num_samples][D]; datum: host i64[num_samples]
 *   (nullable).  compact (nullable, host i64[2][num_samples D]): instead of need_ppf, the inversion's inputs
 *   packed in draw order -- uni[j] the j-th uniform, compact[j] its element index i D + d, compact[num_samples
 *   D + j] its term index datum D + d -- and *n_compact = their count (need_ppf then nullable).
 *   Replaces the scalar draw loop of bohb.py:133-147 (the scoring moved to hbx_kde_acquire). */
int64_t hbx_mt_state_bytes(void);
int hbx_mt_draw(void* state, int32_t kind, int64_t n, int64_t high, double* out);
int hbx_bohb_draw(void* state, const double* data, int64_t n, int32_t D, const double* bw, const int64_t* levels,
                  double bw_factor, int64_t num_samples, double* vals, double* uni, uint8_t* need_ppf,
                  int64_t* datum, int64_t* stop, int64_t* compact, int64_t* n_compact);

#ifdef __cplusplus
}
#endif

#endif /* HBX_H_ */
