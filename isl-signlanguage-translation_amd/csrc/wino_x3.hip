// 3x3 convolution (stride 1, pad 1) as Winograd F(2x2, 3x3) on the gfx950
// FP16 matrix cores with split-fp16 (x3) products -- the fp32-accurate
// arithmetic of conv_x3.hip applied to the 16 Winograd GEMMs:
//
//   V = B^T d B   (4x4 input tile, per channel)        -- fp32 in-kernel, then split
//   U = G g G^T   (per (co, ci), host, double)         -- scaled by 2^s, pre-split
//   M[xi] = sum_ci U[xi][co][ci] V[xi][ci][tile]        -- 16 GEMMs, 3 fp16 MFMAs
//                   (Uh Vh + Uh Vl + Ul Vh, f32 accumulate) per product
//   Y = A^T M A   (2x2 outputs, in registers)
//
// 16 products per 2x2 outputs instead of 36 MACs: 2.25x fewer MFMA FLOPs than
// the direct split-fp16 kernel.  Replaces the 3x3 nn.Conv2d (+ReLU / PReLU)
// layers of src/model.py:25-64 (97 % of body_25's FLOPs).
//
// STATUS: opt-in (ISLPOSE_X3_WINO=1).  Parity-green (rel err 3e-6 vs oracle) but
// 1.3-1.8x slower than conv_x3.hip on every body_25 shape (r01 microbenchmark):
// the transform + split is ~184 VALU ops per (tile, channel) (PMC: 736 VALU per
// wave per step vs 48 MFMAs), i.e. twice the MFMA time it feeds at 64 output
// channels per block, and the 128 KB single-buffered step cannot grow the block.
//
// Block = 4 waves (2 x 2): 64 output channels x 64 tiles (256 outputs); each
// wave owns 32 channels x 32 tiles for ALL 16 xi (16 accumulator tiles, 256
// registers; one wave per SIMD), so the inverse transform is per-lane register
// math (lane l: tile l&31, channels (r&3)+8(r>>2)+4(l>>5) of every xi).
//
// K loop: one step = 16 input channels (a pair of 8-channel chunks); lane half
// h carries chunk h of the pair.  LDS holds one step (single-buffered, 128 KB):
//   U [xi][hi|lo][h][64 co]    x 16 B    -- LDS-DMA from the packed filters
//   V [xi][hi|lo][h][64 tiles] x 16 B    -- transform of the input tile
// Per step:  compute phase  (48 MFMAs per wave from LDS, while the next step's
//            input rows load into registers)
//            write phase    (U DMA issued; V transform + split + ds_write)
// Work item of a thread (its wave's (h, row-half) are uniform): one tile, one
// chunk (8 channels), one row half hf: 3 input rows x 4 columns -> V rows
// 2hf, 2hf+1 (8 of the 16 xi).
#ifdef ISLPOSE_DEV   // measured 1.3-1.8x slower than conv_x3: development builds only
#include <cmath>
#include <type_traits>

#include "internal.h"

namespace isl {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct WinoX3Args {
  const float* in;
  float* out;
  const f16x8* upk;      // [co_tile][pair][xi 16][hi|lo][h][64] x 8 halves
  const float* bias;
  const float* slope;
  int* range_flag;
  long long in_fs, in_chs;      // frame / chunk strides (floats)
  long long out_fs, out_chs;
  float wscale_inv;
  int in_pad, out_pad;
  int H, W, TW, tiles, cin_chunks, pairs, cout, co_tiles, t_tiles, act, nblocks;
};

constexpr int WX_BCO = 64, WX_BT = 64;

__global__ void __launch_bounds__(256, 1) wino_x3_f16(WinoX3Args a) {
  constexpr int BCO = WX_BCO, BT = WX_BT;
  constexpr int US = 16 * 2 * 2 * BCO;          // 16-byte units per U step (64 KB)
  constexpr int VS = 16 * 2 * 2 * BT;           // per V step (64 KB)
  __shared__ f16x8 smem[US + VS];

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
  const int wave_m = wave & 1, wave_n = wave >> 1;
  const int h = lane >> 5, l32 = lane & 31;

  // work item: tile j = lane (64 tiles per wave-instruction), chunk ih, row half hf (wave-uniform)
  const int j = lane;
  const int ih = wave & 1;
  const int hf = __builtin_amdgcn_readfirstlane(wave >> 1);
  int roff[3], coff[4];
  {
    const int tile = min(t0 + j, a.tiles - 1);
    const int ty = tile / a.TW, tx = tile - ty * a.TW;
    // padded input rows 2ty-1+hf+r (+pad), columns 2tx-1+m (+pad); rows / columns past
    // the ring (odd H / W) only feed discarded outputs: clamped
#pragma unroll
    for (int r = 0; r < 3; ++r) roff[r] = min(2 * ty - 1 + hf + r + a.in_pad, Hp - 1) * Wp;
#pragma unroll
    for (int m = 0; m < 4; ++m) coff[m] = min(2 * tx - 1 + m + a.in_pad, Wp - 1);
  }

  f32x4 raw[3][4][2];
  auto load_raw = [&](int t) __attribute__((always_inline)) {
    const int c = min(2 * min(t, a.pairs - 1) + ih, a.cin_chunks - 1);
    const float* src = in_f + (size_t)c * a.in_chs;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float* p = src + (size_t)(roff[r] + coff[m]) * 8;
        raw[r][m][0] = *(const f32x4*)p;
        raw[r][m][1] = *(const f32x4*)(p + 4);
      }
  };
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  auto issue_u = [&](int t) __attribute__((always_inline)) {
    const f16x8* src = a.upk + ((size_t)co_t * a.pairs + t) * US;
#pragma unroll
    for (int k = 0; k < US / 64 / 4; ++k) {
      const int q = wave_u + 4 * k;
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 64 + lane),
                                       (__attribute__((address_space(3))) void*)(smem + q * 64), 16, 0, 0);
    }
  };
  // V transform of the loaded rows for step t, split to fp16 hi / lo, into LDS.
  // rows(): the B^T row combinations, which consume every raw register -- done
  // before the U DMA is issued, so the compiler's wait for the row loads does
  // not also wait for the DMA; cols(): column combinations, split, ds_write.
  f32x4 u[2][4][2];
  auto rows = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if (hf == 0) {   // rows d0 d1 d2: B^T rows 0, 1
          u[0][m][e] = raw[0][m][e] - raw[2][m][e];
          u[1][m][e] = raw[1][m][e] + raw[2][m][e];
        } else {         // rows d1 d2 d3: B^T rows 2, 3
          u[0][m][e] = raw[1][m][e] - raw[0][m][e];
          u[1][m][e] = raw[0][m][e] - raw[2][m][e];
        }
      }
  };
  auto cols = [&](int t) __attribute__((always_inline)) {
    const bool zero = 2 * t + ih >= a.cin_chunks;   // odd chunk count: the pair's 2nd chunk is 0
    f16x8* V = smem + US;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int col = 0; col < 4; ++col) {
        f32x4 v[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          if (col == 0) v[e] = u[q][0][e] - u[q][2][e];
          else if (col == 1) v[e] = u[q][1][e] + u[q][2][e];
          else if (col == 2) v[e] = u[q][2][e] - u[q][1][e];
          else v[e] = u[q][1][e] - u[q][3][e];
        }
        f16x8 hi, lo;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float x = zero ? 0.f : v[k >> 2][k & 3];
          hi[k] = (_Float16)x;
          lo[k] = (_Float16)(x - (float)hi[k]);
        }
        const int xi = 4 * (2 * hf + q) + col;
        V[((xi * 2 + 0) * 2 + ih) * BT + j] = hi;
        V[((xi * 2 + 1) * 2 + ih) * BT + j] = lo;
      }
  };

  f32x16 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

  auto compute = [&]() __attribute__((always_inline)) {
    const f16x8* U = smem + h * BCO + wave_m * 32 + l32;
    const f16x8* V = smem + US + h * BT + wave_n * 32 + l32;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      const f16x8 Ah = U[(x * 2 + 0) * 2 * BCO], Al = U[(x * 2 + 1) * 2 * BCO];
      const f16x8 Bh = V[(x * 2 + 0) * 2 * BT], Bl = V[(x * 2 + 1) * 2 * BT];
      acc[x] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bh, acc[x], 0, 0, 0);
      acc[x] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bl, acc[x], 0, 0, 0);
      acc[x] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Al, Bh, acc[x], 0, 0, 0);
    }
  };

  const int T = a.pairs;
  load_raw(0);
  rows();
  issue_u(0);
  cols(0);
  load_raw(1);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    compute();
    __syncthreads();                    // every wave is done reading step t
    if (t + 1 < T) {
      rows();                           // consumes raw (loaded during step t's compute)
      issue_u(t + 1);
      load_raw(t + 2);                  // next rows in flight across the coming compute phase
      cols(t + 1);
      __syncthreads();                  // vmcnt(0): U landed; V written
    }
  }

  // epilogue: Y = A^T M A per (lane tile, channel), x 2^-s, bias + activation,
  // range check, 2x2 pixel stores (A^T = [1 1 1 0; 0 1 -1 -1])
  const int tile = t0 + wave_n * 32 + l32;
  if (tile >= a.tiles) return;
  const int ty = tile / a.TW, tx = tile - ty * a.TW;
  const int oy = 2 * ty, ox = 2 * tx;
  const int Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int co = co_t * BCO + wave_m * 32 + 8 * q + 4 * h;
    if (co >= a.cout) continue;          // cout % 4 == 0 (host-checked): a group is all in or all out
    f32x4 y[2][2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * q + e;
      float t_[2][4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        t_[0][jj] = acc[0 * 4 + jj][r] + acc[1 * 4 + jj][r] + acc[2 * 4 + jj][r];
        t_[1][jj] = acc[1 * 4 + jj][r] - acc[2 * 4 + jj][r] - acc[3 * 4 + jj][r];
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
      for (int jx = 0; jx < 2; ++jx) {
        if (oy + i >= a.H || ox + jx >= a.W) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = y[i][jx][e] * a.wscale_inv + b[e];
        if (a.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (a.act == ACT_PRELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) bad |= !(__builtin_fabsf(v[e]) < 65504.f);
        *(f32x4*)(out_f + (size_t)(co >> 3) * a.out_chs +
                  (size_t)((oy + i + a.out_pad) * Wo + ox + jx + a.out_pad) * 8 + (co & 7)) = v;
      }
  }
  if (bad) atomicOr(a.range_flag, 1);
}

hipError_t launch_wino_x3(const ConvLaunch& c, hipStream_t s) {
  if (c.ks != 3 || c.in_pad < 1) { set_error("wino_x3: 3x3 with an input ring >= 1 only"); return hipErrorInvalidValue; }
  if (c.cout % 4 != 0) { set_error("wino_x3: cout must be a multiple of 4"); return hipErrorInvalidValue; }
  if ((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) { set_error("wino_x3: slice not on a chunk"); return hipErrorInvalidValue; }
  if (!c.wx3 || !c.range_flag) { set_error("wino_x3: split filters / range flag missing"); return hipErrorInvalidValue; }
  WinoX3Args a;
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  if (a.in_chs >= 0x7fffffffLL) { set_error("wino_x3: frame too large"); return hipErrorInvalidValue; }
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.upk = (const f16x8*)c.wx3; a.bias = c.bias; a.slope = c.slope;
  a.range_flag = c.range_flag;
  a.wscale_inv = c.wscale_inv;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.TW = (c.W + 1) / 2;
  a.tiles = ((c.H + 1) / 2) * a.TW;
  a.cin_chunks = c.cin_chunks;
  a.pairs = (c.cin_chunks + 1) / 2;
  a.cout = c.cout;
  a.co_tiles = (c.cout + WX_BCO - 1) / WX_BCO;
  a.t_tiles = (a.tiles + WX_BT - 1) / WX_BT;
  a.act = c.act;
  const long long nb = (long long)c.n * a.t_tiles * a.co_tiles;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("wino_x3: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  hipLaunchKernelGGL(wino_x3_f16, dim3(a.nblocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

double wino_x3_mfma_flops(const ConvLaunch& c) {
  const double tiles = (double)((c.H + 1) / 2) * ((c.W + 1) / 2);
  return 3.0 * 2.0 * 16 * std::ceil(c.cout / (double)WX_BCO) * WX_BCO * (((c.cin_chunks + 1) / 2) * 16.0) * std::ceil(tiles / WX_BT) * WX_BT * c.n;
}

}  // namespace isl
#endif  // ISLPOSE_DEV
