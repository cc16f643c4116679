/*
 * islpose.h — C ABI of libislpose.so, the MI355X (gfx950) OpenPose keypoint engine.
 *
 * Drop-in boundary for the reference's hot path
 * (sunilsarolkarcds/ISL-SignLanguage-Translation):
 *
 *   module seam  : bodypose_25_model / bodypose_model / handpose_model .forward
 *                  (src/model.py:179-207, 302-329, 394-407), weights loaded through
 *                  util.transfer (src/util.py:35-44)          -> isl_net_create,
 *                  isl_net_set_param, isl_net_forward
 *   frame seam   : Body.__call__ (src/body.py:39-235)         -> isl_net_preprocess
 *                  (one call per pyramid scale) + isl_net_run + isl_body_post
 *                  Hand.__call__ (src/hand.py:24-74)          -> isl_net_preprocess /
 *                  isl_net_preprocess_crops + isl_net_run + isl_hand_post
 *
 * Conventions
 *   - every function returns 0 (ISL_OK) or a negative ISL_E_* code and records a
 *     message retrievable with isl_last_error() (thread-local);
 *   - device pointers are plain HIP device addresses; the caller owns every I/O
 *     buffer, the library owns the weights and an activation arena per net;
 *   - `stream` is a hipStream_t (NULL = default stream); work is stream-ordered,
 *     no function synchronises the device except where noted;
 *   - one isl_net per device; not thread-safe without external locking.
 */
#ifndef ISLPOSE_H
#define ISLPOSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ISL_ABI_VERSION 1

enum isl_kind { ISL_BODY25 = 0, ISL_COCO = 1, ISL_HAND = 2 };

enum isl_status {
  ISL_OK = 0,
  ISL_E_ARG = -1,       /* bad argument / shape                                  */
  ISL_E_PARAM = -2,     /* unknown or missing parameter name (Python: KeyError)  */
  ISL_E_HIP = -3,       /* HIP runtime error                                     */
  ISL_E_CAPACITY = -4,  /* a fixed-capacity result buffer overflowed             */
  ISL_E_STATE = -5,     /* call sequence error (e.g. forward before all params)  */
  ISL_E_INDEX = -6,     /* reference IndexError (3-way subset match, body.py:196)*/
  ISL_E_RANGE = -7      /* split-fp16 conv: an activation reached |x| >= 65504   */
};

/* Convolution arithmetic (all fp32-accurate; not in the reference, which runs
 * torch's fp32 conv):
 *   ISL_ALGO_X3     every conv on the FP16 matrix cores with 3-term operand
 *                   splitting (x*w = xh*wh + xh*wl + xl*wh, fp32 accumulate) --
 *                   the default;
 *   ISL_ALGO_WINO   3x3 convs as Winograd F(2x2,3x3) on the FP32 matrix cores;
 *   ISL_ALGO_DIRECT every conv as a direct implicit GEMM on the FP32 matrix cores. */
enum isl_algo { ISL_ALGO_X3 = 0, ISL_ALGO_WINO = 1, ISL_ALGO_DIRECT = 2 };

typedef struct isl_net isl_net;

int isl_abi_version(void);
const char* isl_last_error(void);

/* ---- module seam --------------------------------------------------------- */

/* Replaces `bodypose_25_model()` / `bodypose_model()` / `handpose_model()`
 * construction (src/model.py:66,210,331) on `device`. */
int isl_net_create(int kind, int device, isl_net** out);
int isl_net_destroy(isl_net* net);

/* Parameter table in caffe naming (the keys of the flat weight dict that
 * util.transfer maps onto state_dict, src/util.py:35-44). */
int isl_net_param_count(const isl_net* net);
int isl_net_param_info(const isl_net* net, int index, const char** name, int64_t* numel);

/* Copy one parameter from host memory (float32, the caffe/torch layout:
 * OIHW for conv weights).  Unknown name or wrong numel -> ISL_E_PARAM.
 * Weights are repacked for the MFMA kernels once all are present. */
int isl_net_set_param(isl_net* net, const char* caffe_name, const float* host, int64_t numel);

/* Replaces `model.forward(x)`: x is float32 NCHW [n,3,h,w] on the device.
 * body25/coco: out0 = PAF [n,npaf,h/8,w/8], out1 = heat [n,njoint,h/8,w/8];
 * hand: out0 = heat [n,22,h/8,w/8], out1 must be NULL.  (floor-mode pooling.) */
int isl_net_forward(isl_net* net, const float* d_x_nchw, int n, int h, int w,
                    float* d_out0, float* d_out1, void* stream);

/* ---- frame seam ---------------------------------------------------------- */

/* Pre-processing of Body/Hand.__call__ for one scale (body.py:53-56):
 * frames uint8 [n,H,W,3] (BGR, device) -> cv2.resize(INTER_CUBIC, fx=fy=scale)
 * -> padRightDownCorner(stride 8, 128) -> float32/256 - 0.5, written straight
 * into the net's input buffer.  Returns the padded net size in *net_h, *net_w. */
int isl_net_preprocess(isl_net* net, const uint8_t* d_frames, int n, int H, int W,
                       double scale, int* net_h, int* net_w, void* stream);

/* A square (or any) sub-image of frame `frame`: pixels [y, y+h) x [x, x+w). */
typedef struct {
  int32_t frame, x, y, w, h;
} isl_crop;

/* Pre-processing of a batch of crops (Hand.__call__ on oriImg[y:y+h, x:x+w],
 * src/hand.py:33-41; demo.py:36): crop i is resized by fx = fy =
 * scale_times_box / h_i (the reference's `scale = x * boxsize / oriImg.shape[0]`)
 * with OpenCV's INTER_CUBIC on the crop as its own image (borders replicated
 * at the crop's edges), padded and normalised into slot i of the net input.
 * Every crop must resize to the same padded net size (true for the hand
 * pyramid: round(s * 368) for every crop width); otherwise ISL_E_ARG. */
int isl_net_preprocess_crops(isl_net* net, const uint8_t* d_frames, int n_frames, int H, int W,
                             const isl_crop* crops, int n_crops, double scale_times_box, int* net_h,
                             int* net_w, void* stream);

/* Run the network on the input buffer filled by isl_net_preprocess; outputs stay
 * in the arena (low-res, 8-channel chunks) for the post kernels, and are also
 * copied to d_out0/d_out1 (NCHW) when those are non-NULL. */
int isl_net_run(isl_net* net, float* d_out0, float* d_out1, void* stream);

/* Activation arenas (not in the reference: torch's caching allocator plays this
 * role there).  A net keeps one arena per net input size (h, w), sized by
 * capacity: a batch of n frames reuses an arena holding n' >= n frames, and a
 * larger n replaces it.  Arenas of other sizes are evicted least-recently-used
 * once the net's arenas would exceed the byte budget (env ISLPOSE_ARENA_BUDGET_MB,
 * default 65536; the arena in use is never evicted).  Reports the bytes held and
 * the number of arenas. */
int isl_net_arena_info(const isl_net* net, int64_t* bytes, int* n_arenas);

/* Select the conv arithmetic of a net (default ISL_ALGO_X3, or the env
 * ISLPOSE_CONV_ALGO=x3|wino|direct at create time). */
int isl_net_set_algo(isl_net* net, int algo);
int isl_net_get_algo(const isl_net* net);

/* K ranges of the ISL_ALGO_X3 convolutions (latency of small grids such as batch-1
 * frames; not in the reference, whose torch conv runs per frame):
 *   mode 1 (default)  canonical ranges: layers of <= 1024 pixels per frame (Mode R's
 *                     23x41 body stages, the 184 px hand scale) sum their input
 *                     channels in up to 8 ranges fixed by the layer shape; a small grid
 *                     spreads the ranges over blocks (split-K, fixed-order reduction),
 *                     a large one keeps them in one block -- the same bits either way,
 *                     so a frame's maps do not depend on the batch it came in;
 *   mode 0            no ranges;
 *   mode 2            latency: mode 1, plus an adaptive split of every other layer
 *                     whose grid cannot half-fill the GPU (those layers' bits then
 *                     depend on the batch size, within the fp32 tolerance).
 * Env ISLPOSE_X3_SPLITK=0|1|2 sets the mode at create time. */
int isl_net_set_split_k(isl_net* net, int mode);

/* Graph replay of the conv chain (not in the reference: it replaces the per-op launches of
 * its torch module, src/model.py:171-207, with one HIP graph launch).  on = 1:
 * the first isl_net_run / isl_net_forward of a run key (batch size, K-range mode, conv
 * algorithm, ISLPOSE_* environment) on an arena runs eagerly, the second captures the
 * launches on a private stream and launches the graph on the caller's stream, later runs
 * replay it -- the same kernels with the same arguments, the same bits.  Timed runs
 * (isl_net_set_timing) stay eager; weight uploads and workspace growth drop the graphs.
 * on = 0 (default; replay measured level at batch 32 and slower at batch 1): every run
 * eager.  Env ISLPOSE_NET_GRAPH=0|1 turns replay off / on process-wide. */
int isl_net_set_graph(isl_net* net, int on);

/* A non-blocking stream for one lane of a pyramid's scales (not in the reference: its scales
 * run one after another on torch's current stream, body.py:47-77 / hand.py:31-50), created
 * with a priority class: -1 the device's greatest priority, 0 the middle of its range, +1 its
 * least.  HIP gives a process a few hardware queues per priority (GPU_MAX_HW_QUEUES, 4 by
 * default) and maps further streams onto them, so two scales on two streams of one priority
 * may still run one after the other; lanes of different priorities never share a queue, and
 * the command processor dispatches the high-priority lane (the largest scale, the critical
 * path) first.  *stream receives a hipStream_t; isl_lane_stream_destroy waits for its work
 * and frees it. */
int isl_lane_stream_create(int device, int priority_class, void** stream);
int isl_lane_stream_destroy(void* stream);

/* Range guard of ISL_ALGO_X3: waits for the device, returns ISL_E_RANGE if any
 * conv output since the last clear left the fp16 split range (the results of
 * those runs are then not fp32-accurate and must be recomputed with
 * ISL_ALGO_DIRECT), else ISL_OK; clear != 0 resets the flag.  The post records
 * of isl_body_post carry the same flag in their status word without a sync. */
int isl_net_check(isl_net* net, int clear);
/* The same check stream-ordered, for pipelined callers: enqueues on `stream` a copy of
 * the flag into *h_flag (pinned host memory; valid once the stream has reached it) and
 * its reset.  *h_flag != 0 then means ISL_E_RANGE for the work enqueued before. */
int isl_net_check_async(isl_net* net, int32_t* h_flag, void* stream);
/* Range-guard diagnostics: *trips = how many checks (isl_net_check with clear != 0, and
 * isl_net_check_async once the stream has reached them) found the flag set, i.e. how
 * many batches the caller had to recompute on the fp32 kernels.  Waits for the device. */
int isl_net_range_info(isl_net* net, int64_t* trips);

/* Per-op device timing (measurement; not in the reference).  After
 * isl_net_set_timing(net, 1) every isl_net_run records a HIP event on its stream
 * before the first op and after each op.  isl_net_timing waits for the recorded
 * runs and returns, per op and summed over them: the duration in ms, the kind
 * (0 max-pool, 1 direct fp32 conv, 2 Winograd conv, 3 split-fp16 conv), the algorithmic FLOPs
 * (2*Cout*Cin*k*k*H*W*n, the direct-convolution count of SURVEY §8d) and the
 * FLOPs the matrix cores executed (tile padding included); then it drops the
 * events.  With op_ms == NULL it only reports *n_ops and *n_runs. */
int isl_net_set_timing(isl_net* net, int on);
int isl_net_timing(isl_net* net, int max_ops, int* n_ops, int* n_runs, double* op_ms, int* op_kind,
                   double* op_flops, double* op_mfma_flops);

/* Diagnostic: the ops of the net's graph (convs by their caffe layer name, pools as
 * "maxpool2") and, for the last isl_net_run / isl_net_forward, which conv kernel variant
 * each ran: for ISL_ALGO_X3 convs the variant code of csrc/internal.h x3_variant_code
 * (VAR bits: 512 row union, 1024 in-block K ranges, 2048 split-K, 4096 two pairs per
 * step, 8192 folds its producers' split-K partials, 32768 pooled-input staging, 65536 one
 * input buffer, 131072 16x16x32 row union, 262144 conv1_1 kernel, 524288 split-K partials
 * left to its consumers (no reduce launch);
 * tile pixels / 32 at bits 20-24, output channels / 32 at bits 25-28, ks / 2 at 29-30);
 * -1 for a pool folded into the next conv's staging; 0 otherwise.  index < the op
 * count (isl_net_timing's *n_ops). */
int isl_net_op_info(const isl_net* net, int index, const char** name, int* variant);

/* Diagnostic: copy the net input buffer (filled by isl_net_preprocess) out as
 * float32 NCHW [n,3,net_h,net_w]. */
int isl_net_debug_input(isl_net* net, float* d_x_nchw, void* stream);

/* Capacities of the per-frame result records. */
typedef struct {
  int32_t max_peaks;   /* per part                                            */
  int32_t max_pairs;   /* candidate (i,j) pairs scored per limb (>= nA*nB)    */
  int32_t max_conns;   /* accepted connections per limb                       */
  int32_t max_rows;    /* subset rows during assembly                         */
} isl_caps;

/* Byte offsets inside one frame's result record (device memory, 8-byte aligned):
 *   int32  status                       ISL_OK / ISL_E_CAPACITY / ISL_E_INDEX
 *   int32  n_peaks[32]                  per part (body: njoint-1 parts)
 *   int32  n_conns[32]                  per limb, -1 = limb skipped (special_k)
 *   int32  n_rows                       subset rows after pruning
 *   double peaks[parts][max_peaks][3]   (x, y, score); id = running count
 *   double conns[limbs][max_conns][5]   (idA, idB, score, i, j)   body.py:171
 *   double subset[max_rows][njoint+1]                             body.py:182-231
 */
typedef struct {
  int64_t status, n_peaks, n_conns, n_rows, peaks, conns, subset, record_bytes;
} isl_layout;

int isl_body_layout(int model_kind, const isl_caps* caps, isl_layout* out);

/* Geometry of one scale of the pyramid (body.py:51-78): the net ran on a padded
 * input of net_h x net_w whose valid (un-padded) part is valid_h x valid_w. */
typedef struct {
  int32_t net_h, net_w;       /* padded net input size (multiples of 8)         */
  int32_t valid_h, valid_w;   /* resized image size before padding              */
} isl_scale_geom;

/* Body post-processing (body.py:64-235) for n frames of size H x W.
 * For each scale s, low-res maps are read from d_paf[s] / d_heat[s] (float32
 * NCHW [n,C,net_h/8,net_w/8]); NULL entries mean "use the net's own arena
 * output" (valid only for nscales == 1, right after isl_net_run).
 * Results: n records of isl_body_layout(...).record_bytes at d_result. */
int isl_body_post(isl_net* net, int n, int H, int W, int nscales, const isl_scale_geom* geom,
                  const float* const* d_paf, const float* const* d_heat,
                  const isl_caps* caps, void* d_result, void* stream);

/* Hand post-processing (hand.py:51-74) for n crops of size h x w: per scale,
 * low-res hand maps (NCHW [n,22,net_h/8,net_w/8], NULL = the net's arena output
 * for nscales == 1) -> int64 peaks [n][21][2] as (x, y), [0, 0] when no pixel of
 * the blurred part map exceeds 0.05. */
int isl_hand_post(isl_net* net, int n, int h, int w, int nscales, const isl_scale_geom* geom,
                  const float* const* d_heat, int64_t* d_peaks, void* stream);

/* Hand post-processing of n square crops of different sizes in one call
 * (HandEstimator.post_crops; hand.py:51-74 per crop): crop i is crop_w[i] px (host
 * array), geom[i*nscales + si] its geometry at scale si (host), its low-res maps crop
 * i of d_heat[si] (NCHW [n,22,net_h/8,net_w/8]; every crop has the same net size per
 * scale) -> int64 peaks [n][21][2].  Stream-ordered on `stream`: the crops run side by
 * side on the net's internal post streams, forked from and joined back into it.  The
 * batch's stage-1 maps live in a buffer of their own whose next writer waits (on the
 * device) for the lanes of the previous call, whatever stream either runs on.
 * Host synchronisation: only when a call needs more lane or stage-1 scratch than any
 * call before it does it wait for that buffer's earlier readers before reallocating
 * (once per new maximum size); otherwise it never blocks the host. */
int isl_hand_post_crops(isl_net* net, int n, const int32_t* crop_w, int nscales,
                        const isl_scale_geom* geom, const float* const* d_heat, int64_t* d_peaks,
                        void* stream);

/* Diagnostic: numpy's np.sum of a float64 array (pairwise 8192-element buffers added
 * left to right, hand.py:68's association) as the hand post computes it for component
 * sums (the block-cooperative device routine): d_out[0] = sum(d_a[0..n)). */
int isl_debug_np_sum(const double* d_a, int64_t n, double* d_out, void* stream);

/* Sign classifier of ISLSignPosTranslator (reference demo_isl_translate.py:72-100,
 * applied in src/ISL_Model_parameter.py:337 to a [1,20,156] window of
 * populate_features rows, :376-443): Masking(0) -> BatchNorm -> BiLSTM(32, seq)
 * -> BiLSTM(32) -> elu -> Dense32 -> BN -> elu -> Dense32 -> BN -> elu ->
 * Dense(n_classes) softmax, inference semantics (dropouts off, keras masking).
 * d_params: float32, the keras `model.get_weights()` list flattened in order
 * (isl_sign_param_count floats); d_windows: float32 [batch][window][n_features];
 * d_probs: float32 [batch][n_classes].  window <= 32, n_features <= 256,
 * n_classes <= 1024.  One workgroup per window, one launch per call. */
int isl_sign_param_count(int n_features, int n_classes, int64_t* count);
int isl_sign_classify(const float* d_params, int n_features, int window, int n_classes,
                      const float* d_windows, int batch, float* d_probs, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ISLPOSE_H */
