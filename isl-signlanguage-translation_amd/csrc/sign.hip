// Sign classifier of ISLSignPosTranslator (reference demo_isl_translate.py:72-100,
// called from src/ISL_Model_parameter.py:337): one workgroup per 20-frame window of
// 156-d keypoint features, the whole keras stack in one launch:
//
//   Masking(0) -> BatchNorm -> Bidirectional(LSTM 32, return_sequences)
//   -> Bidirectional(LSTM 32) -> elu -> Dense 32 -> BN -> elu -> Dense 32 -> BN
//   -> elu -> Dense n_classes + softmax                 (Dropouts: inference no-ops)
//
// Keras semantics kept: a frame is masked when every feature is exactly 0
// (Masking); masked steps carry (h, c) and, in the return_sequences layer, emit
// zeros (Bidirectional sets zero_output_for_mask = return_sequences); the
// backward direction walks the window in reverse and its sequence output is
// stored at the original time index; the mask propagates to the second layer.
// LSTM gates in keras order (i, f, c, o), sigmoid / tanh; BN eps = 1e-3.
//
// Thread map (1024 lanes = 16 waves): lane % 256 = direction * 128 + gate-row.  The
// input projection x_t @ K is split over four step ranges (lane / 256), one pass over
// K each (coalesced over the gate row, x broadcast from LDS); the recurrence (lanes
// < 256) keeps the lane's column of the
// recurrent kernel in 32 VGPRs and needs two barriers per step (gate
// activations, then the 64 (direction, unit) cell updates).  The work is tiny
// (≈2 MFLOP per window) and latency-bound; the point of the kernel is one launch
// per batch of windows instead of hundreds of framework ops.
#include <string>

#include "internal.h"
#include "islpose.h"

namespace isl {

constexpr int SC_U = 32;            // LSTM units (reference: LSTM(32))
constexpr int SC_G = 4 * SC_U;      // gate rows per direction
constexpr int SC_D = 32;            // Dense widths of the head
constexpr int SC_TMAX = 32;         // longest window
constexpr int SC_FMAX = 256;        // widest feature vector
constexpr int SC_CMAX = 1024;       // most classes
constexpr int SC_THREADS = 2 * SC_G;  // lanes of the recurrence: (direction, gate row)
constexpr int SC_BLOCK = 4 * SC_THREADS; // the projections also split the window in 4 step ranges
constexpr int SC_TQT = SC_TMAX / 4;      // steps per range
constexpr float SC_EPS = 1e-3f;     // keras BatchNormalization epsilon

struct SignArgs {
  const float* x;        // [batch, T, F]
  float* out;            // [batch, C] softmax probabilities
  int T, F, C;
  const float* bn0;      // gamma, beta, mean, var  [4][F]
  const float* k1[2];    // [F][4U]
  const float* r1[2];    // [U][4U]
  const float* b1[2];    // [4U]
  const float* k2[2];    // [2U][4U]
  const float* r2[2];
  const float* b2[2];
  const float* d1;       // [2U][D]
  const float* bn1;      // [4][D]
  const float* d2;       // [D][D]
  const float* bn2;      // [4][D]
  const float* d3;       // [D][C]
  const float* b3;       // [C]
};

__device__ __forceinline__ float sc_sigmoid(float z) { return 1.0f / (1.0f + expf(-z)); }
__device__ __forceinline__ float sc_elu(float v) { return v > 0.0f ? v : expm1f(v); }
__device__ __forceinline__ float sc_bn(const float* p, int n, int j, float v) {
  // keras: (x - mean) * rsqrt(var + eps) * gamma + beta
  return (v - p[2 * n + j]) / sqrtf(p[3 * n + j] + SC_EPS) * p[j] + p[n + j];
}

// z[t][d][g] = b[g] + sum_f in[t][f] * K[f][g] (one lane per (d, g, range of 8 steps)).
// A lone window is latency-bound: 1024 lanes on one CU, four K rows per iteration and
// 16-byte LDS reads of the inputs; the sum over f keeps its order.
__device__ void sc_project(const float* in, int F, int T, const float* K, const float* b, int g, int tq,
                           float* zrow) {
  const int tb = tq * SC_TQT;
  if (tb >= T) return;
  float acc[SC_TQT];
  const float bias = b[g];
#pragma unroll
  for (int k = 0; k < SC_TQT; ++k) acc[k] = bias;
  if ((F & 3) == 0) {
#pragma unroll 4
    for (int f = 0; f < F; f += 4) {
      const float w0 = K[(size_t)f * SC_G + g], w1 = K[(size_t)(f + 1) * SC_G + g];
      const float w2 = K[(size_t)(f + 2) * SC_G + g], w3 = K[(size_t)(f + 3) * SC_G + g];
#pragma unroll
      for (int k = 0; k < SC_TQT; ++k)
        if (tb + k < T) {
          const float4 v = *(const float4*)(in + (tb + k) * F + f);
          acc[k] = (((acc[k] + v.x * w0) + v.y * w1) + v.z * w2) + v.w * w3;
        }
    }
  } else {
    for (int f = 0; f < F; ++f) {
      const float w = K[(size_t)f * SC_G + g];
#pragma unroll
      for (int k = 0; k < SC_TQT; ++k)
        if (tb + k < T) acc[k] += in[(tb + k) * F + f] * w;
    }
  }
#pragma unroll
  for (int k = 0; k < SC_TQT; ++k)
    if (tb + k < T) zrow[(tb + k) * SC_THREADS] = acc[k];
}

// One bidirectional LSTM layer over s_z (projected inputs); seq != nullptr writes
// the return_sequences output [T][2U] (zeros at masked steps); h_last gets the
// final (carried) hidden state of each direction.
__device__ void sc_recur(const float* s_z, const int* s_mask, int T, const float* R, int d, int g, int tid,
                         float (*s_h)[SC_U], float (*s_act)[SC_G], float* seq, float* h_last) {
  const bool act = tid < SC_THREADS;     // the other lanes only keep the barriers
  float r[SC_U];
#pragma unroll
  for (int k = 0; k < SC_U; ++k) r[k] = act ? R[k * SC_G + g] : 0.0f;
  const int gate = g / SC_U;
  float c = 0.0f;
  if (tid < 2 * SC_U) s_h[tid / SC_U][tid % SC_U] = 0.0f;
  __syncthreads();
  for (int s = 0; s < T; ++s) {
    if (act) {
      const int t = d == 0 ? s : T - 1 - s;
      float z = s_z[t * SC_THREADS + d * SC_G + g];
#pragma unroll
      for (int k = 0; k < SC_U; ++k) z += s_h[d][k] * r[k];
      s_act[d][g] = gate == 2 ? tanhf(z) : sc_sigmoid(z);
    }
    __syncthreads();
    if (tid < 2 * SC_U) {
      const int dd = tid / SC_U, u = tid % SC_U;
      const int tt = dd == 0 ? s : T - 1 - s;
      float h = 0.0f;
      if (s_mask[tt]) {
        c = s_act[dd][SC_U + u] * c + s_act[dd][u] * s_act[dd][2 * SC_U + u];
        h = s_act[dd][3 * SC_U + u] * tanhf(c);
        s_h[dd][u] = h;
      }
      if (seq) seq[tt * 2 * SC_U + dd * SC_U + u] = h;
    }
    __syncthreads();
  }
  if (tid < 2 * SC_U) h_last[tid] = s_h[tid / SC_U][tid % SC_U];
  __syncthreads();
}

__global__ __launch_bounds__(SC_BLOCK) void sign_classify_kernel(SignArgs a) {
  __shared__ __attribute__((aligned(16))) float s_x[SC_TMAX * SC_FMAX];          // 32 KB: window, then BN'd
  __shared__ float s_z[SC_TMAX * SC_THREADS];       // 32 KB: projected gates
  __shared__ __attribute__((aligned(16))) float s_seq[SC_TMAX * 2 * SC_U];       //  8 KB: layer-1 sequence
  __shared__ float s_h[2][SC_U];
  __shared__ float s_act[2][SC_G];
  __shared__ int s_mask[SC_TMAX];
  __shared__ float s_v[2 * SC_U], s_y[SC_D], s_y2[SC_D];
  __shared__ float s_logit[SC_CMAX];
  __shared__ float s_red[SC_THREADS / 64];

  const int tid = threadIdx.x, lt = tid % SC_THREADS, tq = tid / SC_THREADS;
  const int d = lt / SC_G, g = lt % SC_G;
  const bool hw = tid < SC_THREADS;   // the head's lanes
  const int T = a.T, F = a.F, C = a.C;
  const float* x = a.x + (size_t)blockIdx.x * T * F;

  if (tid < SC_TMAX) s_mask[tid] = 0;
  __syncthreads();
  for (int i = tid; i < T * F; i += SC_BLOCK) {
    const float v = x[i];
    s_x[i] = v;
    if (v != 0.0f) s_mask[i / F] = 1;               // Masking(mask_value=0.)
  }
  __syncthreads();
  for (int i = tid; i < T * F; i += SC_BLOCK) s_x[i] = sc_bn(a.bn0, F, i % F, s_x[i]);
  __syncthreads();

  // layer 1: Bidirectional(LSTM(32, return_sequences=True))
  sc_project(s_x, F, T, a.k1[d], a.b1[d], g, tq, s_z + d * SC_G + g);
  __syncthreads();
  sc_recur(s_z, s_mask, T, a.r1[d], d, g, tid, s_h, s_act, s_seq, s_v);

  // layer 2: Bidirectional(LSTM(32)) over the 64-wide sequence
  sc_project(s_seq, 2 * SC_U, T, a.k2[d], a.b2[d], g, tq, s_z + d * SC_G + g);
  __syncthreads();
  sc_recur(s_z, s_mask, T, a.r2[d], d, g, tid, s_h, s_act, nullptr, s_v);

  // head: elu -> Dense -> BN -> elu -> Dense -> BN -> elu -> Dense + softmax
  if (tid < 2 * SC_U) s_v[tid] = sc_elu(s_v[tid]);
  __syncthreads();
  if (tid < SC_D) {
    float acc = 0.0f;
    for (int i = 0; i < 2 * SC_U; ++i) acc += s_v[i] * a.d1[i * SC_D + tid];
    s_y[tid] = sc_elu(sc_bn(a.bn1, SC_D, tid, acc));
  }
  __syncthreads();
  if (tid < SC_D) {
    float acc = 0.0f;
    for (int i = 0; i < SC_D; ++i) acc += s_y[i] * a.d2[i * SC_D + tid];
    s_y2[tid] = sc_elu(sc_bn(a.bn2, SC_D, tid, acc));
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int c = tid; hw && c < C; c += SC_THREADS) {
    float acc = a.b3[c];
    for (int i = 0; i < SC_D; ++i) acc += s_y2[i] * a.d3[i * C + c];
    s_logit[c] = acc;
    mx = fmaxf(mx, acc);
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (hw && (tid & 63) == 0) s_red[tid / 64] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  __syncthreads();
  float sum = 0.0f;
  for (int c = tid; hw && c < C; c += SC_THREADS) {
    const float e = expf(s_logit[c] - mx);
    s_logit[c] = e;
    sum += e;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (hw && (tid & 63) == 0) s_red[tid / 64] = sum;
  __syncthreads();
  sum = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
  float* out = a.out + (size_t)blockIdx.x * C;
  for (int c = tid; hw && c < C; c += SC_THREADS) out[c] = s_logit[c] / sum;
}

// Offsets of keras `model.get_weights()` (Sequential order) in the flat buffer.
static int64_t sign_layout(int F, int C, SignArgs* a, const float* p) {
  int64_t o = 0;
  auto take = [&](int64_t n) { const float* q = p ? p + o : nullptr; o += n; return q; };
  const float* bn0 = take(4LL * F);
  const float *k1[2], *r1[2], *b1[2], *k2[2], *r2[2], *b2[2];
  for (int d = 0; d < 2; ++d) { k1[d] = take((int64_t)F * SC_G); r1[d] = take(SC_U * SC_G); b1[d] = take(SC_G); }
  for (int d = 0; d < 2; ++d) { k2[d] = take(2 * SC_U * SC_G); r2[d] = take(SC_U * SC_G); b2[d] = take(SC_G); }
  const float* d1 = take(2 * SC_U * SC_D);
  const float* bn1 = take(4 * SC_D);
  const float* d2 = take(SC_D * SC_D);
  const float* bn2 = take(4 * SC_D);
  const float* d3 = take((int64_t)SC_D * C);
  const float* b3 = take(C);
  if (a) {
    a->bn0 = bn0; a->d1 = d1; a->bn1 = bn1; a->d2 = d2; a->bn2 = bn2; a->d3 = d3; a->b3 = b3;
    for (int d = 0; d < 2; ++d) {
      a->k1[d] = k1[d]; a->r1[d] = r1[d]; a->b1[d] = b1[d];
      a->k2[d] = k2[d]; a->r2[d] = r2[d]; a->b2[d] = b2[d];
    }
  }
  return o;
}

}  // namespace isl

using namespace isl;

extern "C" int isl_sign_param_count(int n_features, int n_classes, int64_t* count) {
  if (n_features <= 0 || n_features > SC_FMAX || n_classes <= 0 || n_classes > SC_CMAX || !count) {
    set_error("isl_sign_param_count: n_features must be in [1, 256] and n_classes in [1, 1024]");
    return ISL_E_ARG;
  }
  *count = sign_layout(n_features, n_classes, nullptr, nullptr);
  return ISL_OK;
}

extern "C" int isl_sign_classify(const float* d_params, int n_features, int window, int n_classes,
                                 const float* d_windows, int batch, float* d_probs, void* stream) {
  if (batch == 0) return ISL_OK;
  if (!d_params || !d_windows || !d_probs || batch < 0 || window <= 0 || window > SC_TMAX || n_features <= 0 ||
      n_features > SC_FMAX || n_classes <= 0 || n_classes > SC_CMAX) {
    set_error("isl_sign_classify: bad argument (window <= 32, n_features <= 256, n_classes <= 1024)");
    return ISL_E_ARG;
  }
  SignArgs a{};
  a.x = d_windows;
  a.out = d_probs;
  a.T = window;
  a.F = n_features;
  a.C = n_classes;
  sign_layout(n_features, n_classes, &a, d_params);
  hipLaunchKernelGGL(sign_classify_kernel, dim3(batch), dim3(SC_BLOCK), 0, (hipStream_t)stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("sign_classify_kernel: ") + hipGetErrorString(e));
    return ISL_E_HIP;
  }
  return ISL_OK;
}
