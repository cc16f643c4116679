// Direct convolution (3x3 / 1x1 / 7x7, stride 1, "same" padding) as an
// implicit GEMM on the gfx950 FP32 matrix cores (v_mfma_f32_32x32x2_f32).
//
// Replaces every nn.Conv2d (+ReLU / PReLU) of src/model.py:25-64 (make_layers,
// make_layers_Mconv).  FP32 in, FP32 accumulate: each MFMA is an exact fmaf
// chain, so results differ from torch-CPU only by summation order.
//
// GEMM view:  D[co][px] = sum_k Wt[co][k] * X[k][px],  k = (ky, kx, ci).
//   A operand (32 rows)  = 32 output channels      (lane: co = l&31, k = l>>5)
//   B operand (32 cols)  = 32 output pixels        (lane: px = l&31, k = l>>5)
//   D                    = lane holds pixel l&31, channels (r&3)+8(r>>2)+4(l>>5)
//
// Pixel tiles: BPX consecutive output pixels of one frame in raster order
// (flattened M; a frame's last tile is partial, nothing else is wasted).  The
// input buffer is stored in 8-channel chunks with a zero ring (Act.pad >= k/2),
// so in its padded linear pixel index L = (y+p)*(W+2p) + (x+p) the input row dy
// of a whole tile is ONE contiguous segment [La + dy*Wp - P, Lb + dy*Wp + P] of
// 32-byte pixels: no bounds checks, no im2col, fully coalesced loads.
//
// K loop: one step = (8-channel chunk, kernel row ky): stage that row's input
// segment (8 ch) and the KS x 8 x BCO weight slab into LDS (register-staged,
// double-buffered, one barrier per step), then KS taps x 4 MFMA k-steps.
// The 8 channels of a chunk are split in two planes of 4 (ci 0-3 | 4-7); lane
// half h reads plane h with one ds_read_b128 and feeds its 4 floats to 4
// successive MFMAs, so MFMA k-step e covers channels {e, 4+e}.
#include <cmath>

#include "internal.h"

namespace isl {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ConvArgs {
  const float* in;
  float* out;
  const float* wpk;
  const float* bias;
  const float* slope;
  long long in_fs, in_chs;      // frame / chunk strides (floats) of the input buffer
  long long out_fs, out_chs;
  int in_pad, out_pad;
  int H, W, cin_chunks, cout, co_tiles, px_tiles, tpx, act, nblocks;
};

template <int KS, int WAVES_M, int WAVES_N, int WM, int WN, bool GLDS>
// 4 waves per SIMD (4 blocks of 256 threads per CU, <= 128 VGPR+AGPR, <= 40 KB LDS
// each): the 46x82 stage layers (960 tiles at batch 32) then fit in one round.
__global__ void __launch_bounds__(WAVES_M * WAVES_N * 64, 4)
conv_mfma_f32(ConvArgs a) {
  constexpr int NPL = 2;                        // planes of 4 channels per 8-channel chunk
  constexpr int NT = WAVES_M * WAVES_N * 64;
  constexpr int BCO = WAVES_M * WM * 32;
  constexpr int BPX = WAVES_N * WN * 32;
  constexpr int P = KS / 2;
  constexpr int SEGMAX = 2 * BPX;               // input segment capacity (host-checked)
  constexpr int WTILE = KS * NPL * BCO;         // float4 per weight slab (one kernel row)
  constexpr int ACT_IT = (SEGMAX + NT - 1) / NT;
  constexpr int W_IT = (WTILE + NT - 1) / NT;
  constexpr int BUF = NPL * SEGMAX + WTILE;     // float4 per LDS stage
  __shared__ f32x4 smem[2 * BUF];

  // XCD-aware tile order: consecutive logical tiles (the co-tiles of one pixel
  // tile, then neighbouring pixel tiles) land on the same XCD / L2.
  int bid = blockIdx.x;
  {
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int co_t = bid % a.co_tiles;
  const int rest = bid / a.co_tiles;
  const int pt = rest % a.px_tiles;
  const int n = rest / a.px_tiles;

  const int HW = a.H * a.W;
  const int m0 = pt * a.tpx;                    // tpx = BPX unless the image is very narrow
  const int mlast = min(m0 + a.tpx, HW) - 1;
  const int Wi = a.W + 2 * a.in_pad;
  const int ya = m0 / a.W, xa = m0 - ya * a.W;
  const int yb = mlast / a.W, xb = mlast - yb * a.W;
  const int La = (ya + a.in_pad) * Wi + xa + a.in_pad;
  const int Lb = (yb + a.in_pad) * Wi + xb + a.in_pad;
  const int seg = Lb - La + 2 * P + 1;
  const float* in_f = a.in + (size_t)n * a.in_fs;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_m = wave % WAVES_M, wave_n = wave / WAVES_M;
  const int h = lane >> 5, l32 = lane & 31;

  int rel[WN];
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int j = (wave_n * WN + wn) * 32 + l32;
    const int m = min(m0 + j, mlast);
    const int y = m / a.W, x = m - y * a.W;
    rel[wn] = (y + a.in_pad) * Wi + x + a.in_pad - La;
  }

  const int T = a.cin_chunks * KS;
  f32x4 ra[NPL][ACT_IT];
  f32x4 rw[W_IT];

  auto gload = [&](int t) {
    const int c = t / KS, ky = t - c * KS;
    const float* src = in_f + (size_t)c * a.in_chs + (size_t)(La + (ky - P) * Wi - P) * 8;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int i = 0; i < ACT_IT; ++i) {
        const int px = tid + i * NT;
        ra[pl][i] = (px < seg) ? *(const f32x4*)(src + (size_t)px * 8 + 4 * pl) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    const f32x4* wsrc = (const f32x4*)a.wpk + ((size_t)(co_t * a.cin_chunks + c) * KS + ky) * WTILE;
#pragma unroll
    for (int i = 0; i < W_IT; ++i) {
      const int idx = tid + i * NT;
      if (WTILE % NT == 0 || idx < WTILE) rw[i] = wsrc[idx];
    }
  };
  auto lstore = [&](int buf) {
    f32x4* s = smem + buf * BUF;
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int i = 0; i < ACT_IT; ++i) {
        const int px = tid + i * NT;
        if (SEGMAX % NT == 0 || px < SEGMAX) s[pl * SEGMAX + px] = ra[pl][i];
      }
#pragma unroll
    for (int i = 0; i < W_IT; ++i) {
      const int idx = tid + i * NT;
      if (WTILE % NT == 0 || idx < WTILE) s[NPL * SEGMAX + idx] = rw[i];
    }
  };

  // LDS-DMA staging (global_load_lds_dwordx4): every wave-instruction fills 1 KiB
  // of LDS lane-linearly (64 pixels of one channel plane, or 64 float4 of the
  // weight slab), no staging VGPRs and no ds_write; the barrier's vmcnt(0) retires it.
  constexpr int NWAVES = WAVES_M * WAVES_N;
  const int wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto issue = [&](int t, int buf) {
    const int c = t / KS, ky = t - c * KS;
    const float* src = in_f + (size_t)c * a.in_chs + (size_t)(La + (ky - P) * Wi - P) * 8;
    f32x4* s = smem + buf * BUF;
    const int nchunk = (seg + 63) >> 6;
    for (int q = wave_u; q < NPL * nchunk; q += NWAVES) {
      const int pl = q / nchunk, ch = q - pl * nchunk;
      const int px = min(ch * 64 + lane, seg - 1);
      __builtin_amdgcn_global_load_lds((const void*)(src + (size_t)px * 8 + 4 * pl),
                                       (__attribute__((address_space(3))) void*)(s + pl * SEGMAX + ch * 64), 16, 0,
                                       0);
    }
    const f32x4* wsrc = (const f32x4*)a.wpk + ((size_t)(co_t * a.cin_chunks + c) * KS + ky) * WTILE;
    for (int qq = wave_u; qq < WTILE / 64; qq += NWAVES)
      __builtin_amdgcn_global_load_lds((const void*)(wsrc + qq * 64 + lane),
                                       (__attribute__((address_space(3))) void*)(s + NPL * SEGMAX + qq * 64), 16, 0,
                                       0);
  };

  f32x16 acc[WM][WN];
#pragma unroll
  for (int wm = 0; wm < WM; ++wm)
#pragma unroll
    for (int wn = 0; wn < WN; ++wn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[wm][wn][r] = 0.f;

  if constexpr (GLDS) {
    issue(0, 0);
  } else {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const int buf = t & 1;
    if constexpr (GLDS) {
      if (t + 1 < T) issue(t + 1, buf ^ 1);
    } else {
      if (t + 1 < T) gload(t + 1);
    }
    const f32x4* sa = smem + buf * BUF + h * SEGMAX;
    const f32x4* sw = smem + buf * BUF + NPL * SEGMAX + h * BCO + wave_m * WM * 32 + l32;
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) {
      f32x4 A[WM], B[WN];
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) A[wm] = sw[kx * NPL * BCO + wm * 32];
#pragma unroll
      for (int wn = 0; wn < WN; ++wn) B[wn] = sa[rel[wn] + kx];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int wm = 0; wm < WM; ++wm)
#pragma unroll
          for (int wn = 0; wn < WN; ++wn)
            acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[wm][e], B[wn][e], acc[wm][wn], 0, 0, 0);
    }
    if constexpr (!GLDS) {
      if (t + 1 < T) lstore(buf ^ 1);
    }
    __syncthreads();
  }

  // epilogue: bias + activation, masked float4 stores into the output slice
  const int Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int m = m0 + (wave_n * WN + wn) * 32 + l32;
    if (m > mlast) continue;
    const int y = m / a.W, x = m - y * a.W;
    float* op = out_f + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8;
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) {
      const int cob = co_t * BCO + (wave_m * WM + wm) * 32 + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = cob + 8 * q;
        const f32x4 b = *(const f32x4*)(a.bias + co);
        f32x4 v = {acc[wm][wn][4 * q] + b[0], acc[wm][wn][4 * q + 1] + b[1],
                   acc[wm][wn][4 * q + 2] + b[2], acc[wm][wn][4 * q + 3] + b[3]};
        if (a.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (a.act == ACT_PRELU) {
          const f32x4 sl = *(const f32x4*)(a.slope + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
        }
        float* oc = op + (size_t)(co >> 3) * a.out_chs + (co & 7);
        if (co + 3 < a.cout) {
          *(f32x4*)oc = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (co + e < a.cout) oc[e] = v[e];
        }
      }
    }
  }
}

// Staging variant: register staging (default) or LDS-DMA (ISLPOSE_CONV_STAGING=glds).
// Measured equal at batch 32 (122.2 vs 122.4 TF over the net run, r01), so the
// register path stays the default; the DMA path frees 25 VGPRs for larger tiles.
static bool conv_staging_glds() {
  const char* e = getenv("ISLPOSE_CONV_STAGING");
  return e && e[0] == 'g';
}

int conv_bco_for(int cout) {
  if (cout % 128 == 0) return 128;
  if (cout == 96) return 96;
  if (cout > 96) return 128;
  if (cout > 32) return 64;
  return 32;
}

template <int KS, int WAVES_M, int WAVES_N, int WM, int WN>
static hipError_t launch_t(const ConvLaunch& c, hipStream_t s) {
  constexpr int BCO = WAVES_M * WM * 32;
  constexpr int BPX = WAVES_N * WN * 32;
  constexpr int P = KS / 2;
  if (c.in_pad < P) { set_error("conv: input ring narrower than kernel radius"); return hipErrorInvalidValue; }
  constexpr int SEGCAP = 2 * BPX;
  if (c.bco != BCO) { set_error("conv: tile mismatch"); return hipErrorInvalidValue; }
  if ((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) { set_error("conv: slice not on a chunk"); return hipErrorInvalidValue; }
  ConvArgs a;
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.wpk = c.wpk; a.bias = c.bias; a.slope = c.slope;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.cin_chunks = c.cin_chunks; a.cout = c.cout;
  a.co_tiles = (c.cout + BCO - 1) / BCO;
  a.tpx = tile_pixels(c, BPX, SEGCAP);
  a.px_tiles = (c.H * c.W + a.tpx - 1) / a.tpx;
  a.act = c.act;
  const long long nb = (long long)c.n * a.px_tiles * a.co_tiles;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("conv: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  if (conv_staging_glds())
    hipLaunchKernelGGL((conv_mfma_f32<KS, WAVES_M, WAVES_N, WM, WN, true>), dim3(a.nblocks),
                       dim3(WAVES_M * WAVES_N * 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv_mfma_f32<KS, WAVES_M, WAVES_N, WM, WN, false>), dim3(a.nblocks),
                       dim3(WAVES_M * WAVES_N * 64), 0, s, a);
  return hipGetLastError();
}

template <int KS>
static hipError_t launch_ks(const ConvLaunch& c, hipStream_t s) {
  switch (c.bco) {
    case 128: return launch_t<KS, 2, 2, 2, 2>(c, s);
    case 96: return launch_t<KS, 1, 4, 3, 1>(c, s);
    case 64: return launch_t<KS, 1, 4, 2, 1>(c, s);
    case 32: return launch_t<KS, 1, 4, 1, 1>(c, s);
  }
  set_error("conv: unsupported tile");
  return hipErrorInvalidValue;
}

double conv_mfma_flops(const ConvLaunch& c) {
  const int BPX = 128;      // every tile shape above covers 128 pixels
  const double co = (double)((c.cout + c.bco - 1) / c.bco) * c.bco;
  const double px = std::ceil((double)c.H * c.W / tile_pixels(c, BPX, 2 * BPX)) * BPX;
  return 2.0 * co * (c.cin_chunks * 8.0) * c.ks * c.ks * px * c.n;
}

hipError_t launch_conv(const ConvLaunch& c, hipStream_t s) {
  switch (c.ks) {
    case 1: return launch_ks<1>(c, s);
    case 3: return launch_ks<3>(c, s);
    case 7: return launch_ks<7>(c, s);
  }
  set_error("conv: unsupported kernel size");
  return hipErrorInvalidValue;
}

}  // namespace isl
