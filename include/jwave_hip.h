/*
 * jwave_hip.h — C ABI of libjwave_hip.so, the MI355X (gfx950) engine for
 * JWave's FWT / WPT / MODWT convolve-decimate hot path.
 *
 * This is the boundary a JNI shim (or ctypes / cgo / N-API) binds.  Plain C
 * types only: pointers, sizes, ints.  Each entry point names the reference
 * interface it replaces (paths under /root/reference/src/main/java/jwave/).
 *
 * Conventions
 *  - Return value: JWV_OK (0) or an error code; the message (the reference's
 *    exception text where one exists) is in jwv_last_error(ctx).
 *  - Host-pointer entry points (no suffix) copy to the device, compute and copy
 *    back; they return when the result is in `y`.
 *  - `_dev` entry points take device pointers and are asynchronous on the
 *    context's stream (jwv_ctx_set_stream); call jwv_ctx_synchronize or sync
 *    the stream before reading results.  `y` must not overlap `x`.
 *  - Inputs are never modified and pointers are not retained after return
 *    (the reference never mutates inputs: FastWaveletTransform.java:85,
 *    WaveletPacketTransform.java:86-88, MODWTTransform.java:288).
 *  - Arrays are row-major and contiguous unless an `ld` is given.
 *  - Thread safety: a context serialises its own calls with a mutex; use one
 *    context per thread for concurrency (the reference transforms are
 *    stateless and called concurrently: ParallelTransform.java:258-270).
 */
#ifndef JWAVE_HIP_H
#define JWAVE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JWV_OK 0
/* Invalid input that the reference reports with JWaveFailure (length not 2^p,
 * level out of range): FastWaveletTransform.java:74-83,122-131,
 * WaveletPacketTransform.java:76-84,144-152. */
#define JWV_ERR_FAILURE 1
/* MODWT level checks that the reference reports with IllegalArgumentException
 * (MODWTTransform.java:257-282). */
#define JWV_ERR_ILLEGAL_ARGUMENT 2
/* Device / runtime failure (HIP error, out of memory): maps to JWaveError. */
#define JWV_ERR_DEVICE 3
/* Null pointer, bad tap table, overlapping buffers, size beyond int range. */
#define JWV_ERR_BAD_CALL 4

/* Math modes.  EXACT: a*b+c rounded twice, reference summation order — results
 * are bit-identical to the JVM's.  FMA: fused multiply-add (one rounding) in
 * the same order; differs from EXACT by ~1 ulp per tap. */
#define JWV_MATH_EXACT 0
#define JWV_MATH_FMA 1

#define JWV_MAX_TAPS 64

/* A filter bank, read once from the Wavelet getters
 * (transforms/wavelets/Wavelet.java:152-219). */
typedef struct jwv_taps {
  int32_t mother_wavelength;    /* L = getMotherWavelength(), 2..64 */
  int32_t transform_wavelength; /* getTransformWavelength(), normally 2 */
  const double* lo;             /* getScalingDeComposition()   (L doubles) */
  const double* hi;             /* getWaveletDeComposition()   (L doubles) */
  const double* lo_r;           /* getScalingReConstruction()  (L doubles) */
  const double* hi_r;           /* getWaveletReConstruction()  (L doubles) */
  /* 1.0, or 0.5 for Haar1Orthogonal whose reverse() scales every synthesis
   * term (transforms/wavelets/haar/Haar1Orthogonal.java:39,175-207). */
  double reverse_scale;
} jwv_taps;

typedef struct jwv_ctx jwv_ctx;

/* ---- context -------------------------------------------------------------- */
int jwv_ctx_create(int device, jwv_ctx** out);
int jwv_ctx_destroy(jwv_ctx* ctx);
/* Last error message of this context ("" if none).  ctx may be NULL: then the
 * calling thread's last context-less error (e.g. from jwv_ctx_create). */
const char* jwv_last_error(const jwv_ctx* ctx);
/* Launch on a caller-owned hipStream_t (NULL = the legacy default stream);
 * jwv_ctx_reset_stream returns to the context's own non-blocking stream
 * (the default after jwv_ctx_create).  Switching streams makes the new stream
 * wait (an event, no host sync) for the work the context queued on the old
 * one, so its workspace and fused-tail counter stay ordered. */
int jwv_ctx_set_stream(jwv_ctx* ctx, void* hip_stream);
int jwv_ctx_reset_stream(jwv_ctx* ctx);
void* jwv_ctx_get_stream(const jwv_ctx* ctx);
int jwv_ctx_set_math(jwv_ctx* ctx, int mode);
/* Pass plan for single long 1-D FWT signals (no reference counterpart; the
 * results are bit-identical under every plan).  0 = the multi-launch plan.
 * JWV_PLAN_REV_HEAD: the reverse's resident part and first tiled pass in one
 * launch (no inter-workgroup wait: every block recomputes the resident part);
 * JWV_PLAN_CHAIN_REV / _FWD: the whole reverse / forward in one launch (the
 * reverse chain has bounded in-kernel waits, see jwv_ctx_synchronize).
 * JWV_PLAN_FWD_TAIL: the forward's deep tiled pass and its resident pass in
 * one launch (the unit that completes an arrival counter runs the resident
 * levels; no wait).
 * Default: JWV_PLAN_REV_HEAD | JWV_PLAN_FWD_TAIL (jwv_ctx_set_plan is the only
 * way to change it; the library reads no environment setting but the
 * JWV_LAUNCH_LOG diagnostic). */
#define JWV_PLAN_CHAIN_REV 1
#define JWV_PLAN_CHAIN_FWD 2
#define JWV_PLAN_REV_HEAD 4
#define JWV_PLAN_FWD_TAIL 8
int jwv_ctx_set_plan(jwv_ctx* ctx, int flags);
/* Waits for the context's stream.  Also reports (JWV_ERR_DEVICE) a chained
 * launch whose bounded in-kernel wait gave up since the last check (its results
 * are then invalid; only possible if its grid was not co-resident).  The
 * host-pointer entry points make the same check before they return. */
int jwv_ctx_synchronize(jwv_ctx* ctx);
/* Diagnostic: bound of each in-kernel wait in polls (0 = default 2^22).  A
 * tiny bound forces the timeout path (tests of the error contract). */
int jwv_ctx_set_poll_limit(jwv_ctx* ctx, unsigned spins);
/* Profiling: when enabled, every kernel launch is bracketed by a pair of
 * hipEvents recorded on the launch stream.  profile_read synchronises, sums the
 * event times per kernel kind (fwt_fwd_tile, fwt_rev_res, ...), clears the
 * records and fills up to max_out entries; *n_out = number of kinds seen.
 * `bytes` is the algorithmic HBM traffic of those launches. */
typedef struct jwv_kernel_stat {
  char name[32];
  int64_t launches;
  double total_ms;
  double bytes;
} jwv_kernel_stat;
int jwv_ctx_profile_enable(jwv_ctx* ctx, int on);
int jwv_ctx_profile_read(jwv_ctx* ctx, jwv_kernel_stat* out, int max_out, int* n_out);
/* Restrict profiling events to one kernel kind (by name; NULL or "" = all). */
int jwv_ctx_profile_select(jwv_ctx* ctx, const char* kind);
/* Release cached device workspace and the pinned staging ring.
 * A context owns its workspace and its fused-tail arrival counters: it runs
 * one transform at a time (calls on one context are serialised), and a stream
 * switch orders the new stream after the old one (jwv_ctx_set_stream).  Work
 * other code queues on the old stream after the switch is not ordered before
 * the context's next launch.  Footprint: device workspace as large as the largest
 * transform's intermediates (one matrix for 2-D / 3-D), plus, once a host
 * entry staged pageable memory, 4 x 32 MiB of pinned host memory; the host
 * copy threads are one process-wide pool. */
int jwv_ctx_trim(jwv_ctx* ctx);

/* Page-locked host memory for the host-pointer entry points.  The host entry
 * points (no _dev suffix) stage pageable arrays through a pinned ring in
 * chunks (host copies overlapped with the DMA); arrays that are already
 * page-locked -- from jwv_host_alloc, hipHostMalloc or hipHostRegister -- are
 * DMA'd directly.  The JNI shim copies Java arrays into such a buffer with
 * Get/SetDoubleArrayRegion instead of holding a critical region across the
 * GPU work.  No Java counterpart (boundary plumbing). */
int jwv_host_alloc(jwv_ctx* ctx, int64_t bytes, void** p);
int jwv_host_free(jwv_ctx* ctx, void* p);
/* Cumulative seconds the context's host entries spent staging pageable
 * arrays: out[0] host copies into the pinned ring, out[1] waits for a ring
 * slot's H2D DMA, out[2] waits for a slot's D2H DMA, out[3] host copies out
 * of the ring, out[4] bytes staged in, out[5] bytes staged out.  reset != 0
 * zeroes them after reading.  Diagnostic (bench.py's host_entry object). */
int jwv_ctx_stage_stats(jwv_ctx* ctx, double* out6, int reset);
/* Threads of the process-wide host copy pool that stages pageable arrays
 * (counting the calling thread): min(CPU affinity, 16) for single-device use,
 * grown to min(CPU affinity, 16 x devices) by jwv_mctx_create. */
int jwv_host_copy_threads(void);
int jwv_version(void);

/* ---- 1-D FWT ---------------------------------------------------------------
 * FastWaveletTransform.forward(double[], int level)  FastWaveletTransform.java:71-101
 * FastWaveletTransform.reverse(double[], int level)  FastWaveletTransform.java:119-153
 * (full depth, WaveletTransform.forward/reverse(double[]) :77-112, is
 *  level = log2(n)). */
int jwv_fwt_fwd_f64(const double* x, double* y, int64_t n, int level, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_fwt_rev_f64(const double* y, double* x, int64_t n, int level, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_fwt_fwd_f64_dev(const double* x, double* y, int64_t n, int level, const jwv_taps* t,
                        jwv_ctx* ctx);
int jwv_fwt_rev_f64_dev(const double* y, double* x, int64_t n, int level, const jwv_taps* t,
                        jwv_ctx* ctx);

/* Batched 1-D FWT: `batch` independent signals of length n, signal b at
 * x + b*ld (ld >= n); the same for y.  Equivalent to one forward(double[],
 * level) per signal (the batch loop of ParallelizationOpportunityTest.java:80-98). */
int jwv_fwt_fwd_batch_f64(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                          int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_rev_batch_f64(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                          int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_fwd_batch_f64_dev(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                              int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_rev_batch_f64_dev(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                              int level, const jwv_taps* t, jwv_ctx* ctx);

/* ---- segmented row passes (sharded 2-D FWT) -------------------------------
 * The row pass of the 2-D FWT (BasicTransform.java:369-378 forward, :461-470
 * reverse): `rows` rows of length cols, level `level` each, with the
 * coefficient side in the all-to-all layout of the sharded 2-D transform
 * (jwave_amd/distributed.py): chunk j = columns [j*seg, (j+1)*seg) of every
 * row, stored [cols/seg][rows][seg].  fwd: x plain [rows][cols] -> y chunked;
 * rev: y chunked -> x plain.  seg: a power of two >= 2 dividing cols.  Results
 * are those of jwv_fwt_{fwd,rev}_batch_f64_dev on the plain layout, value for
 * value; device pointers only, x and y must not overlap.  Where the row
 * kernels cannot address the chunks (short rows, seg < 1024) the entry runs the
 * plain pass and a packing copy. */
int jwv_fwt_rows_seg_fwd_f64_dev(const double* x, double* y, int64_t rows, int64_t cols,
                                 int level, int64_t seg, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_rows_seg_rev_f64_dev(const double* y, double* x, int64_t rows, int64_t cols,
                                 int level, int64_t seg, const jwv_taps* t, jwv_ctx* ctx);

/* ---- multi-device batches ---------------------------------------------------
 * One context per listed device (duplicates allowed).  The batched host
 * entries split the batch into contiguous blocks of signals, device i taking
 * signals [start_i, start_i + count_i) of jwv_batch_split(batch, n, i), and
 * run the blocks concurrently, one host thread per device (stage in,
 * transform, stage out on that device's stream): no collective, every device
 * its own PCIe link.  They return when every device has finished; arguments
 * are validated once, with the single-device messages, before any device
 * starts; a device failure returns that device's status and message
 * (jwv_mctx_last_error; the lowest failing device index wins).  Results are
 * those of the single-device batched entries, signal for signal.
 * Reference: the executor over independent signals of
 * src/test/java/jwave/ParallelizationOpportunityTest.java:80-98, spread over the
 * node's GPUs. */
typedef struct jwv_mctx jwv_mctx;
int jwv_mctx_create(const int* devices, int n_devices, jwv_mctx** out);
int jwv_mctx_destroy(jwv_mctx* m);
const char* jwv_mctx_last_error(const jwv_mctx* m);
int jwv_mctx_size(const jwv_mctx* m);
/* the per-device context i (profiling, streams, trim); owned by m */
jwv_ctx* jwv_mctx_ctx(jwv_mctx* m, int i);
int jwv_mctx_set_math(jwv_mctx* m, int mode);
/* Contiguous block of device i (0 <= i < n_devices) in a batch of `batch`:
 * start = floor(batch*i/n), count = floor(batch*(i+1)/n) - start.  Pure
 * arithmetic, no device needed. */
int jwv_batch_split(int64_t batch, int n_devices, int i, int64_t* start, int64_t* count);
int jwv_m_fwt_fwd_batch_f64(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                            int level, const jwv_taps* t, jwv_mctx* m);
int jwv_m_fwt_rev_batch_f64(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                            int level, const jwv_taps* t, jwv_mctx* m);
int jwv_m_wpt_fwd_batch_f64(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                            int level, const jwv_taps* t, jwv_mctx* m);
int jwv_m_wpt_rev_batch_f64(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                            int level, const jwv_taps* t, jwv_mctx* m);
/* ParallelTransform.forward / reverse(double[][], lvlM, lvlN)
 * (ParallelTransform.java:70-126) over the listed devices: device i takes the
 * row block [i rw, (i+1) rw) and, after one device-to-device exchange
 * (hipMemcpyPeerAsync over xGMI), the column slab [i cw, (i+1) cw), rw =
 * rows/D, cw = cols/D: forward = H2D row block, row pass straight into the
 * exchange layout, exchange, column pass, D2H of the column slab into the host
 * matrix's columns; reverse mirrors it.  D = the largest power of two <= the
 * device count that divides rows with cw >= 2 (1: the single-device entry on
 * device 0).  Host arrays as jwv_fwt2d_*_f64; results are that entry's bits.
 * Distinct physical devices have not been measured on this project's 1-GPU
 * pool (tests list device 0 twice). */
int jwv_m_fwt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m);
int jwv_m_fwt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m);
int jwv_m_wpt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m);
int jwv_m_wpt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m);
/* MODWTTransform.forwardMODWT / inverseMODWT of `batch` signals of length n
 * (MODWTTransform.java:256-375): x [batch][n], coefficients [batch][J+1][n]
 * (each signal's double[J+1][n] packed).  jwv_modwt_*_batch_f64 on one
 * device, signal after signal; jwv_m_*: contiguous blocks of signals per
 * device (jwv_batch_split), one host thread per device.  Validation and
 * messages are forwardMODWT's. */
int jwv_modwt_fwd_batch_f64(const double* x, double* wv, int64_t batch, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* ctx);
int jwv_modwt_inv_batch_f64(const double* wv, double* x, int64_t batch, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* ctx);
int jwv_m_modwt_fwd_batch_f64(const double* x, double* wv, int64_t batch, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m);
int jwv_m_modwt_inv_batch_f64(const double* wv, double* x, int64_t batch, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m);

/* ---- 2-D / 3-D FWT -----------------------------------------------------------
 * BasicTransform.forward(double[][], lvlM, lvlN)  BasicTransform.java:361-399
 *   (rows with lvlN, then columns with lvlM); reverse :436-474 (columns, then
 *   rows).  x is rows*cols row-major (a JNI shim packs double[][] rows).
 * BasicTransform.forward(double[][][], lvlP, lvlQ, lvlR)  :509-560 — slice
 *   [i][.][.] gets the 2-D transform with (lvlP, lvlQ), then the lines along i
 *   get lvlR; reverse :602-659.  x is P*Q*R row-major. */
int jwv_fwt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                      int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                      int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt2d_fwd_f64_dev(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                          int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt2d_rev_f64_dev(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                          int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt3d_fwd_f64(const double* x, double* y, int64_t p, int64_t q, int64_t r, int lvl_p,
                      int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt3d_rev_f64(const double* y, double* x, int64_t p, int64_t q, int64_t r, int lvl_p,
                      int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt3d_fwd_f64_dev(const double* x, double* y, int64_t p, int64_t q, int64_t r,
                          int lvl_p, int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt3d_rev_f64_dev(const double* y, double* x, int64_t p, int64_t q, int64_t r,
                          int lvl_p, int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
/* ParallelTransform.reverse(double[][][], lvlP, lvlQ, lvlR)
 * (ParallelTransform.java:183-216) in ONE call: the P axis first (lvlR,
 * Space3DTransformTask :386-394), then each slice's 2-D reverse (columns
 * lvlP, rows lvlQ).  BasicTransform.reverse (:602-659) runs the slices first,
 * so the two orders round differently; ParallelTransform.forward equals
 * BasicTransform.forward and uses jwv_fwt3d_fwd_f64. */
int jwv_fwt3d_rev_pt_f64(const double* y, double* x, int64_t p, int64_t q, int64_t r, int lvl_p,
                         int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt3d_rev_pt_f64_dev(const double* y, double* x, int64_t p, int64_t q, int64_t r,
                             int lvl_p, int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);

/* ---- CompressorMagnitude / denoise ---------------------------------------------
 * CompressorMagnitude(threshold).compress(double[])
 * (compressions/CompressorMagnitude.java:73-84, Compressor.java:96-110):
 * y[i] = |x[i]| >= m * threshold ? x[i] : 0 with m = sum|x| / n.  A threshold
 * <= 0 becomes 1.0 (Compressor.java:66-80).  y equals Java's output for
 * every input: m is summed as a fixed tree, and only when some |x[i]| lies in
 * the tree sum's n*eps band around the cut is Java's left-to-right sum formed
 * on the device and used instead.  magnitude: optional host pointer for m
 * (the tree value, or Java's when the left-to-right pass ran).  x == y (in
 * place) is allowed; partially overlapping x and y are JWV_ERR_BAD_CALL.
 * jwv_fwt_denoise_*: forward(level) -> compress -> reverse(level) without
 * leaving the device (the Transform + Compressor denoising sequence). */
int jwv_compress_magnitude_f64(const double* x, double* y, int64_t n, double threshold,
                               double* magnitude, jwv_ctx* ctx);
int jwv_compress_magnitude_f64_dev(const double* x, double* y, int64_t n, double threshold,
                                   double* magnitude, jwv_ctx* ctx);
int jwv_fwt_denoise_f64(const double* x, double* y, int64_t n, int level, double threshold,
                        const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_denoise_f64_dev(const double* x, double* y, int64_t n, int level, double threshold,
                            const jwv_taps* t, jwv_ctx* ctx);

/* ---- one axis of a block -------------------------------------------------------
 * The per-dimension pass inside BasicTransform's 2-D/3-D loops
 * (BasicTransform.java:369-395 rows / columns, :520-558 lines along i): the
 * FWT (or WPT) of every line along the middle axis of a contiguous
 * [outer][len][inner] block.  Rows: inner = 1; columns of a slab: outer = 1.
 * Device pointers only; used by the sharded 2-D transform (column pass on a
 * [rows][cols/W] slab after the all-to-all). */
int jwv_fwt_axis_fwd_f64_dev(const double* x, double* y, int64_t outer, int64_t len,
                             int64_t inner, int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_fwt_axis_rev_f64_dev(const double* y, double* x, int64_t outer, int64_t len,
                             int64_t inner, int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt_axis_fwd_f64_dev(const double* x, double* y, int64_t outer, int64_t len,
                             int64_t inner, int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt_axis_rev_f64_dev(const double* y, double* x, int64_t outer, int64_t len,
                             int64_t inner, int level, const jwv_taps* t, jwv_ctx* ctx);

/* ---- WPT ---------------------------------------------------------------------
 * WaveletPacketTransform.forward(double[], int level)  WaveletPacketTransform.java:73-124
 * WaveletPacketTransform.reverse(double[], int level)  WaveletPacketTransform.java:141-191
 * (same math: PooledWaveletPacketTransform, ParallelWaveletPacketTransform). */
int jwv_wpt_fwd_f64(const double* x, double* y, int64_t n, int level, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_wpt_rev_f64(const double* y, double* x, int64_t n, int level, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_wpt_fwd_f64_dev(const double* x, double* y, int64_t n, int level, const jwv_taps* t,
                        jwv_ctx* ctx);
int jwv_wpt_rev_f64_dev(const double* y, double* x, int64_t n, int level, const jwv_taps* t,
                        jwv_ctx* ctx);
int jwv_wpt_fwd_batch_f64(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                          int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt_rev_batch_f64(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                          int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt_fwd_batch_f64_dev(const double* x, double* y, int64_t batch, int64_t n, int64_t ld,
                              int level, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt_rev_batch_f64_dev(const double* y, double* x, int64_t batch, int64_t n, int64_t ld,
                              int level, const jwv_taps* t, jwv_ctx* ctx);
/* 2-D / 3-D packet transforms through the same BasicTransform loops. */
int jwv_wpt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                      int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                      int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt2d_fwd_f64_dev(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                          int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt2d_rev_f64_dev(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                          int lvl_n, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt3d_fwd_f64(const double* x, double* y, int64_t p, int64_t q, int64_t r, int lvl_p,
                      int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
int jwv_wpt3d_rev_f64(const double* y, double* x, int64_t p, int64_t q, int64_t r, int lvl_p,
                      int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);
/* ParallelTransform(WaveletPacketTransform).reverse 3-D order (see
 * jwv_fwt3d_rev_pt_f64) */
int jwv_wpt3d_rev_pt_f64(const double* y, double* x, int64_t p, int64_t q, int64_t r, int lvl_p,
                         int lvl_q, int lvl_r, const jwv_taps* t, jwv_ctx* ctx);

/* ---- AncientEgyptianDecomposition / decompose ----------------------------------
 * transform: which BasicTransform is wrapped. */
#define JWV_TRANSFORM_FWT 0 /* FastWaveletTransform */
#define JWV_TRANSFORM_WPT 1 /* WaveletPacketTransform */
/* AncientEgyptianDecomposition(transform).forward / reverse(double[])
 * (transforms/AncientEgyptianDecomposition.java:97-184): any length n >= 1 is
 * split into power-of-two pieces (MathToolKit.decompose, largest first,
 * tools/MathToolKit.java:57-80), each transformed at full depth in place.
 * Every piece <= 8192 samples runs in ONE varlen launch. */
int jwv_aed_fwd_f64(const double* x, double* y, int64_t n, int transform, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_aed_rev_f64(const double* y, double* x, int64_t n, int transform, const jwv_taps* t,
                    jwv_ctx* ctx);
int jwv_aed_fwd_f64_dev(const double* x, double* y, int64_t n, int transform,
                        const jwv_taps* t, jwv_ctx* ctx);
int jwv_aed_rev_f64_dev(const double* y, double* x, int64_t n, int transform,
                        const jwv_taps* t, jwv_ctx* ctx);
/* WaveletTransform.decompose(double[]) (transforms/WaveletTransform.java:136-145):
 * mat receives (log2(n)+1) rows of n, row p = forward(x, p).  recompose(mat,
 * level) (:173-182) is jwv_fwt_rev_f64 / jwv_wpt_rev_f64 on row `level`. */
int jwv_decompose_f64(const double* x, double* mat, int64_t n, int transform,
                      const jwv_taps* t, jwv_ctx* ctx);
int jwv_decompose_f64_dev(const double* x, double* mat, int64_t n, int transform,
                          const jwv_taps* t, jwv_ctx* ctx);

/* ---- MODWT -------------------------------------------------------------------
 * MODWTTransform.forwardMODWT(double[] data, int maxLevel)  MODWTTransform.java:256-306
 *   wv receives (J+1)*n doubles, row-major [W_1 .. W_J, V_J] (coeffs[0..J]).
 *   DIRECT circular convolution semantics (:677-690).
 * MODWTTransform.inverseMODWT(double[][] coefficients)     MODWTTransform.java:337-375
 *   wv as produced by the forward; J = coefficients.length - 1. */
int jwv_modwt_fwd_f64(const double* x, double* wv, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* ctx);
int jwv_modwt_inv_f64(const double* wv, double* x, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* ctx);
int jwv_modwt_fwd_f64_dev(const double* x, double* wv, int64_t n, int J, const jwv_taps* t,
                          jwv_ctx* ctx);
int jwv_modwt_inv_f64_dev(const double* wv, double* x, int64_t n, int J, const jwv_taps* t,
                          jwv_ctx* ctx);
/* The same on coefficient rows at a stride ldw >= n doubles (row j at
 * wv + j*ldw): the sharded MODWT (jwave_amd/distributed.py) keeps a slice's
 * rows between halo columns and transforms them in place of a packed copy.
 * No reference counterpart (the reference's double[][] rows are ldw = n). */
int jwv_modwt_fwd_ld_f64_dev(const double* x, double* wv, int64_t ldw, int64_t n, int J,
                             const jwv_taps* t, jwv_ctx* ctx);
int jwv_modwt_inv_ld_f64_dev(const double* wv, int64_t ldw, double* x, int64_t n, int J,
                             const jwv_taps* t, jwv_ctx* ctx);
/* The MODWT filters g, h (L doubles each) the engine derives from t
 * (MODWTTransform.initializeFilterCache :452-484). Host-only, no device. */
int jwv_modwt_filters(const jwv_taps* t, double* g, double* h);

#ifdef __cplusplus
}
#endif
#endif /* JWAVE_HIP_H */
