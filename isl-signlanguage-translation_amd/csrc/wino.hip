// 3x3 convolution (stride 1, pad 1) as fused Winograd F(2x2, 3x3) on the gfx950
// FP32 matrix cores.  Replaces the 3x3 nn.Conv2d (+ReLU / PReLU) layers of
// src/model.py:25-64 -- 97 % of body_25's FLOPs -- with 16 small GEMMs per
// 2x2 output tile instead of 36 MACs per output pixel (2.25x fewer MFMA flops).
// All arithmetic is fp32 (transforms on the VALU, products on
// v_mfma_f32_32x32x2_f32); results differ from the direct convolution by
// rounding only, well inside the 1e-4 relative tolerance of north_star.
//
//   V = B^T d B   (4x4 input tile d, per channel)      -- in-kernel, into LDS
//   U = G g G^T   (3x3 filter g, per (co, ci))        -- host, at weight upload
//   M[xi] = sum_ci U[xi][co][ci] V[xi][ci][tile]       -- 16 GEMMs on the MFMA
//   Y = A^T M A   (2x2 outputs)                        -- in registers
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  A^T = [1 1 1 0; 0 1 -1 -1]
//
// Block = WAVES_M x WAVES_N waves; each wave owns 32 output channels x 32 tiles
// for ALL 16 xi (16 accumulator tiles, 256 registers), so the inverse transform
// is per-lane register math: lane l holds tile l&31, channels (r&3)+8(r>>2)+4(l>>5)
// of every xi.  One wave per SIMD.
//
// K loop: one step = one 8-channel chunk.  U[xi][plane][co] (float4 = 4 channels
// of a plane) arrives by LDS-DMA; V[xi][plane][tile] is computed from 3 input
// rows per (tile, plane, row-half) work item held in registers since the
// previous step.  Double-buffered, one barrier per step; per step and wave:
// 16 xi x 4 k-steps = 64 MFMAs from 32 ds_read_b128.
#include <cmath>
#include <type_traits>

#include "internal.h"

namespace isl {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct WinoArgs {
  const float* in;
  float* out;
  const float* upk;      // [co_tile][chunk][xi 16][plane 2][BCO][4]
  const float* bias;
  const float* slope;
  long long in_fs, in_chs;      // frame / chunk strides (floats), see Act
  long long out_fs, out_chs;
  int in_pad, out_pad;
  int H, W, TW, tiles, cin_chunks, co_tiles, t_tiles, act, nblocks;
};

template <int WAVES_M, int WAVES_N>
__global__ void __launch_bounds__(WAVES_M * WAVES_N * 64, 1) wino_f23_mfma(WinoArgs a) {
  constexpr int NT = WAVES_M * WAVES_N * 64;
  constexpr int NWAVES = WAVES_M * WAVES_N;
  constexpr int BCO = WAVES_M * 32;
  constexpr int BT = WAVES_N * 32;
  constexpr int UT = 16 * 2 * BCO;            // float4 per U stage
  constexpr int VT = 16 * 2 * BT;             // float4 per V stage
  constexpr int ITEMS = BT * 4;               // (tile, plane, row half) per stage
  constexpr int IPT = (ITEMS + NT - 1) / NT;
  static_assert(UT % 64 == 0, "U stage is whole 1 KiB DMA pieces");
  __shared__ f32x4 smem[2 * (UT + VT)];

  int bid = blockIdx.x;
  {
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int co_t = bid % a.co_tiles;
  const int rest = bid / a.co_tiles;
  const int pt = rest % a.t_tiles;
  const int n = rest / a.t_tiles;
  const int t0 = pt * BT;

  const int Hp = a.H + 2 * a.in_pad, Wp = a.W + 2 * a.in_pad;
  const float* in_f = a.in + (size_t)n * a.in_fs;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_m = wave % WAVES_M, wave_n = wave / WAVES_M;
  const int h = lane >> 5, l32 = lane & 31;

  // transform work items of this thread: item = tid + i*NT -> tile j, plane pl, half hf
  // (threads past ITEMS redo an item: same values to the same LDS words, no branch)
  int roff[IPT][3], coff[IPT][4], vdst[IPT];
  int hf_of[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    const int it = (tid + i * NT) % ITEMS;
    const int j = it % BT, pl = (it / BT) & 1, hf = it / (2 * BT);
    hf_of[i] = hf;
    const int tile = min(t0 + j, a.tiles - 1);
    const int ty = tile / a.TW, tx = tile - ty * a.TW;
    // padded input rows 2ty-1+k (+pad), k = hf..hf+2; columns 2tx-1+m (+pad), m = 0..3.
    // Rows / columns past the ring (odd H / W) only feed discarded outputs: clamped.
#pragma unroll
    for (int r = 0; r < 3; ++r) roff[i][r] = min(2 * ty - 1 + hf + r + a.in_pad, Hp - 1) * Wp;
#pragma unroll
    for (int m = 0; m < 4; ++m) coff[i][m] = min(2 * tx - 1 + m + a.in_pad, Wp - 1);
    vdst[i] = (2 * hf * 4) * 2 * BT + pl * BT + j;   // xi = 4*(2hf) + 0 row of V
  }
  int cpl[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) cpl[i] = ((((tid + i * NT) % ITEMS) / BT) & 1) * 4;

  typedef f32x4 Raw[IPT][3][4];
  const int T = a.cin_chunks;
  f32x16 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;
  auto load_raw = [&](Raw& raw, int c) __attribute__((always_inline)) {
    c = min(c, T - 1);   // past the end: harmless reload (its V is never read)
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int m = 0; m < 4; ++m)
          raw[i][r][m] = *(const f32x4*)(in_f + (size_t)c * a.in_chs + (size_t)(roff[i][r] + coff[i][m]) * 8 + cpl[i]);
    }
  };
  constexpr int NP = 9 * IPT;
  static_assert(IPT <= 2, "at most two transform items per thread");
  static_assert((UT / 64) % NWAVES == 0, "U stage splits evenly over the waves");
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_u = [&](int c, int buf) __attribute__((always_inline)) {
    c = min(c, T - 1);
    const f32x4* src = (const f32x4*)a.upk + (size_t)(co_t * a.cin_chunks + c) * UT;
    f32x4* dst = smem + buf * (UT + VT);
#pragma unroll
    for (int k = 0; k < UT / 64 / NWAVES; ++k) {
      const int q = wave_u + k * NWAVES;
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 64 + lane),
                                       (__attribute__((address_space(3))) void*)(dst + q * 64), 16, 0, 0);
    }
  };

  // The K loop, instantiated per row-half pattern HFM (bit i = half of item i),
  // which is uniform over a wave: the transform is straight-line code.
  auto kloop = [&](auto hfm_c) __attribute__((always_inline)) {
    constexpr int HFM = decltype(hfm_c)::value;
    // V transform of one work item in 9 pieces: piece 0 = the two B^T rows (over
    // 4 columns), pieces 1..8 = one V float4 each (row q, column col) + ds_write.
    f32x4 u[IPT][2][4];
    auto put_piece = [&](Raw& raw, int buf, int i, int p) __attribute__((always_inline)) {
      if (p == 0) {
        if (((HFM >> i) & 1) == 0) {    // raw rows d0 d1 d2: B^T rows 0, 1
#pragma unroll
          for (int m = 0; m < 4; ++m) { u[i][0][m] = raw[i][0][m] - raw[i][2][m]; u[i][1][m] = raw[i][1][m] + raw[i][2][m]; }
        } else {                        // raw rows d1 d2 d3: B^T rows 2, 3
#pragma unroll
          for (int m = 0; m < 4; ++m) { u[i][0][m] = raw[i][1][m] - raw[i][0][m]; u[i][1][m] = raw[i][0][m] - raw[i][2][m]; }
        }
        return;
      }
      const int q = (p - 1) >> 2, col = (p - 1) & 3;
      const f32x4* x = u[i][q];
      f32x4 v;
      if (col == 0) v = x[0] - x[2];
      else if (col == 1) v = x[1] + x[2];
      else if (col == 2) v = x[2] - x[1];
      else v = x[1] - x[3];
      smem[buf * (UT + VT) + UT + vdst[i] + q * 4 * 2 * BT + col * 2 * BT] = v;
    };

    // One K step: MFMAs over buffer `buf` (chunk t).  Chunk t+1's filters
    // (LDS-DMA) and input rows (registers) are issued first; its V transform is
    // woven between the MFMAs of the second half of the step, by which time the
    // rows have landed.  The closing barrier retires everything for step t+1.
    // (Loading the rows two steps ahead with the transform from the first slot,
    // or issuing the loads between the MFMAs, both measured slower: r01.)
    Raw raw;
    auto step = [&](int t, int buf) __attribute__((always_inline)) {
      issue_u(t + 1, buf ^ 1);
      load_raw(raw, t + 1);
      const f32x4* U = smem + buf * (UT + VT) + h * BCO + wave_m * 32 + l32;
      const f32x4* V = smem + buf * (UT + VT) + UT + h * BT + wave_n * 32 + l32;
      // 8 slots of two xi each; the two accumulation chains alternate so that no
      // MFMA waits on the one just issued.
      f32x4 A0 = U[0], B0 = V[0], A1 = U[2 * BCO], B1 = V[2 * BT];
#pragma unroll
      for (int x = 0; x < 16; x += 2) {
        f32x4 A0n = A0, B0n = B0, A1n = A1, B1n = B1;
        if (x < 14) {
          A0n = U[(x + 2) * 2 * BCO];
          B0n = V[(x + 2) * 2 * BT];
          A1n = U[(x + 3) * 2 * BCO];
          B1n = V[(x + 3) * 2 * BT];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[e], B0[e], acc[x], 0, 0, 0);
          acc[x + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[e], B1[e], acc[x + 1], 0, 0, 0);
        }
        if (x >= 8) {           // transform pieces in the last 4 slots, once the rows have landed
          const int sl = x / 2 - 4;
#pragma unroll
          for (int p = sl * NP / 4; p < (sl + 1) * NP / 4; ++p) put_piece(raw, buf ^ 1, p / 9, p % 9);
        }
        A0 = A0n; B0 = B0n; A1 = A1n; B1 = B1n;
        __builtin_amdgcn_sched_barrier(0);   // keep the weave: no hoisting of later slots' reads
      }
      __syncthreads();
    };

    issue_u(0, 0);
    load_raw(raw, 0);
#pragma unroll
    for (int p = 0; p < NP; ++p) put_piece(raw, 0, p / 9, p % 9);
    __syncthreads();
    for (int t = 0; t < T; t += 2) {
      step(t, 0);
      if (t + 1 < T) step(t + 1, 1);
    }
  };
  if constexpr (IPT == 1) {
    if (__builtin_amdgcn_readfirstlane(hf_of[0]) == 0) kloop(std::integral_constant<int, 0>{});
    else kloop(std::integral_constant<int, 1>{});
  } else {
    kloop(std::integral_constant<int, 2>{});   // item 0 in the upper half, item 1 in the lower
  }

  // epilogue: Y = A^T M A per (lane tile, channel), bias + activation, 2x2 pixel stores
  const int tile = t0 + wave_n * 32 + l32;
  if (tile >= a.tiles) return;
  const int ty = tile / a.TW, tx = tile - ty * a.TW;
  const int oy = 2 * ty, ox = 2 * tx;
  const int Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int co = co_t * BCO + wave_m * 32 + 8 * q + 4 * h;
    f32x4 y[2][2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * q + e;
      float t_[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t_[0][j] = acc[0 * 4 + j][r] + acc[1 * 4 + j][r] + acc[2 * 4 + j][r];
        t_[1][j] = acc[1 * 4 + j][r] - acc[2 * 4 + j][r] - acc[3 * 4 + j][r];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        y[i][0][e] = t_[i][0] + t_[i][1] + t_[i][2];
        y[i][1][e] = t_[i][1] - t_[i][2] - t_[i][3];
      }
    }
    const f32x4 b = *(const f32x4*)(a.bias + co);
    f32x4 sl = {0.f, 0.f, 0.f, 0.f};
    if (a.act == ACT_PRELU) sl = *(const f32x4*)(a.slope + co);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (oy + i >= a.H || ox + j >= a.W) continue;
        f32x4 v = y[i][j] + b;
        if (a.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (a.act == ACT_PRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
        }
        *(f32x4*)(out_f + (size_t)(co >> 3) * a.out_chs + (size_t)((oy + i + a.out_pad) * Wo + ox + j + a.out_pad) * 8 +
                  (co & 7)) = v;
      }
  }
}

int wino_bco_for(int cout) {
  if (cout % 64 == 0) return 64;
  if (cout % 96 == 0) return 96;
  return 0;   // not eligible: direct kernel
}

template <int WAVES_M, int WAVES_N>
static hipError_t launch_w(const ConvLaunch& c, hipStream_t s) {
  constexpr int BCO = WAVES_M * 32, BT = WAVES_N * 32;
  if (c.ks != 3 || c.in_pad < 1) { set_error("wino: 3x3 with an input ring >= 1 only"); return hipErrorInvalidValue; }
  if (c.cout % BCO != 0 || c.bco != BCO) { set_error("wino: tile mismatch"); return hipErrorInvalidValue; }
  if ((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) { set_error("wino: slice not on a chunk"); return hipErrorInvalidValue; }
  WinoArgs a;
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  if (a.in_chs >= 0x7fffffffLL) { set_error("wino: frame too large"); return hipErrorInvalidValue; }
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.upk = c.wpk; a.bias = c.bias; a.slope = c.slope;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.TW = (c.W + 1) / 2;
  a.tiles = ((c.H + 1) / 2) * a.TW;
  a.cin_chunks = c.cin_chunks;
  a.co_tiles = c.cout / BCO;
  a.t_tiles = (a.tiles + BT - 1) / BT;
  a.act = c.act;
  const long long nb = (long long)c.n * a.t_tiles * a.co_tiles;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("wino: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  hipLaunchKernelGGL((wino_f23_mfma<WAVES_M, WAVES_N>), dim3(a.nblocks), dim3(WAVES_M * WAVES_N * 64), 0, s, a);
  return hipGetLastError();
}

double wino_mfma_flops(const ConvLaunch& c) {
  const double BT = c.bco == 96 ? 32 : 64;
  const double tiles = (double)((c.H + 1) / 2) * ((c.W + 1) / 2);
  return 2.0 * 16 * c.cout * (c.cin_chunks * 8.0) * std::ceil(tiles / BT) * BT * c.n;
}

hipError_t launch_wino(const ConvLaunch& c, hipStream_t s) {
  switch (c.bco) {
    case 64: return launch_w<2, 2>(c, s);
    case 96: return launch_w<3, 1>(c, s);
  }
  set_error("wino: unsupported tile");
  return hipErrorInvalidValue;
}

}  // namespace isl
