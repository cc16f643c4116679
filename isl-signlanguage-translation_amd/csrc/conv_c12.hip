// conv1_1 -> conv1_2 -> the 2x2 pool in one launch, on the split-fp16
// ("x3") matrix-core arithmetic of conv_x3.hip.
//
// Replaces model.py:25-45's first two layers of every net (conv1_1 3 -> 64 + ReLU, conv1_2 64 ->
// 64 + ReLU, pool1_stage1): body_25 (model.py:75-80), COCO and hand.  Unfused, conv1_1 is bound by
// writing its 64-channel fp32 output at full resolution (2 GB per Mode N step at batch 32, ~4 TB/s)
// and conv1_2 reads it back with its halo.  Here a block computes a 2-D tile of conv1_2's output
// (8 rows x 32 columns) and first recomputes conv1_1 on the tile's 10 x 34 halo straight into LDS
// as conv1_2's split B operand (1.33x conv1_1's 27-term products, ~1.6 % of conv1_2's), so
// conv1_1's output never reaches HBM.
//
// Bits: the same as conv_x3_rgb followed by conv_x3_f16 (the 64-channel generic loop).
//   conv1_1: the rgb kernel's K packing (k = 9 ky + 3 kx + c padded to 32, two K steps) and MFMA
//            order, its epilogue (x 2^-s, bias, activation), zero outside the image (conv1_2's
//            padding ring), then x3_split8's split of every value;
//   conv1_2: K order (pair, ky, kx), 3 MFMAs per tap (hi*hi, hi*lo, lo*hi) from zero, its
//            epilogue, then the pool's maxima (pool2: the pooled map; else the hpool pair-max
//            buffer that vpool2 / the next conv's staging finishes).
// Channel halves: conv1_1's 64 outputs are staged 32 at a time (chunk pairs 0-1, then 2-3) so
// the halo buffer is 45 KB and two blocks fit a CU; conv1_2 walks its pairs in order across the
// two halves, so its K order is unchanged.
#include <algorithm>

#include "internal.h"

namespace isl {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int TH = 8, TW = 32;                  // output tile (rows x columns): one row per wave
constexpr int HH = TH + 2, HWD = TW + 2;        // conv1_1 halo of the tile
constexpr int HPX = HH * HWD;                   // 340 halo pixels
constexpr int HG = (HPX + 31) / 32;             // 11 groups of 32 halo pixels (conv1_1 MFMA tiles)
constexpr int HPS = HG * 32;                    // halo plane stride in the LDS buffer (352)
constexpr int NT = 512;                         // 8 waves
constexpr int WSL = 3 * 2 * 2 * 64;             // conv1_2 weight slab of one (pair, ky) step, 16-B units

struct C12Args {
  const float* in;                              // [n][1 chunk][H + 2 p][W + 2 p][8], channels 0-2
  long long in_fs;
  int in_pad;
  const f16x8* w1;                              // pack_x3_rgb: [kk][hi|lo][h][64]
  const float* b1;
  const float* sl1;
  float s1_inv;
  int act1;
  const f16x8* w2;                              // pack_x3 (64-channel tile): [pair][ky][kx][hi|lo][h][64]
  const float* b2;
  const float* sl2;
  float s2_inv;
  int act2;
  float* out;                                   // pool2: the pooled buffer [n][8 chunks][H/2 + 2 op][W/2 + 2 op][8];
  long long out_fs, out_chs;                    // else the pair-max buffer [n][8 chunks][H][W / 2][8]
  int pool2, out_pad, out_wp;                   // out_wp: padded pooled width W/2 + 2 out_pad
  int H, W, tiles_x, tiles_y, nblocks;
  int* range_flag;
};

// x3_split8's arithmetic on 4 values: hi = (f16) x (RNE), lo = (f16) (x - (f32) hi)
__device__ __forceinline__ void split4(const f32x4& a, f16x4& hi, f16x4& lo) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const f32x2 x = f32x2{a[2 * k], a[2 * k + 1]};
    const f16x2 h = __builtin_convertvector(x, f16x2);
    const f32x2 hf = __builtin_convertvector(h, f32x2);
    f32x2 r;
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r.x) : "v"(x.x), "v"(hf.x));
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r.y) : "v"(x.y), "v"(hf.y));
    const f16x2 l = __builtin_convertvector(r, f16x2);
    hi[2 * k] = h.x; hi[2 * k + 1] = h.y;
    lo[2 * k] = l.x; lo[2 * k + 1] = l.y;
  }
}

// RR: both layers ReLU (the VGG conv1 pair of every net), a compile-time activation: the
// run-time test per value made a scalar branch chain of both epilogues
template <bool RR>
__device__ __forceinline__ float act_f(float v, int act, float slope) {
  if (RR || act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_PRELU) return v >= 0.f ? v : v * slope;
  return v;
}

template <bool RR>
__global__ void __launch_bounds__(NT, 4) conv_x3_c12(C12Args a) {
  __shared__ f16x8 s_x[2][4][HPS];              // conv1_1 output half: [hi|lo][chunk of the half][halo px]
  __shared__ f16x8 s_w[2][WSL];                 // conv1_2 weight slabs, double-buffered
  __shared__ float s_p[256];                    // b1, b2, slopes1, slopes2
  __shared__ f32x4 s_in[TH + 4][TW + 4];        // the tile's input rows y0-2 .. y0+TH+1 (channels 0-3)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  int bid = blockIdx.x;
  {   // XCD-aware order (conv_x3_f16): neighbouring tiles, which share halo rows, on one L2
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int tx = bid % a.tiles_x, rest = bid / a.tiles_x;
  const int ty = rest % a.tiles_y, n = rest / a.tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;
  const int Wp = a.W + 2 * a.in_pad, Hp = a.H + 2 * a.in_pad;
  const float* in_f = a.in + (size_t)n * a.in_fs;
  for (int i = tid; i < 64; i += NT) {
    s_p[i] = a.b1[i];
    s_p[64 + i] = a.b2[i];
    s_p[128 + i] = a.act1 == ACT_PRELU ? a.sl1[i] : 0.f;
    s_p[192 + i] = a.act2 == ACT_PRELU ? a.sl2[i] : 0.f;
  }
  // conv1_2 weight slab of step s (pair s / 3, kernel row s % 3): register-staged one step ahead
  // (loads at the step's top, LDS stores at its end), so the load latency hides behind the
  // step's MFMAs; an LDS-DMA slab would be drained at once (hipcc orders every LDS read after
  // an LDS-DMA in flight)
  f16x8 wreg[2];
  auto load_w = [&](int st) __attribute__((always_inline)) {
    const f16x8* src = a.w2 + (size_t)st * WSL;
    wreg[0] = src[tid];
    if (tid < WSL - NT) wreg[1] = src[NT + tid];
  };
  auto store_w = [&](int b) __attribute__((always_inline)) {
    s_w[b][tid] = wreg[0];
    if (tid < WSL - NT) s_w[b][NT + tid] = wreg[1];
  };
  load_w(0);
  store_w(0);
  // the input region every halo pixel's 3 x 3 neighbourhood reads, once for both channel halves
  // (clamped into the padded plane: only out-of-image halo pixels, zeroed below, read the clamps)
  for (int i = tid; i < (TH + 4) * (TW + 4); i += NT) {
    const int ry = i / (TW + 4), rx = i - ry * (TW + 4);
    const int yy = min(max(y0 - 2 + ry + a.in_pad, 0), Hp - 1);
    const int xx = min(max(x0 - 2 + rx + a.in_pad, 0), Wp - 1);
    s_in[ry][rx] = *(const f32x4*)(in_f + ((size_t)yy * Wp + xx) * 8);
  }
  bool bad = false;
  f32x16 acc2[2];
#pragma unroll
  for (int wm = 0; wm < 2; ++wm)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[wm][r] = 0.f;

  for (int hf = 0; hf < 2; ++hf) {
    __syncthreads();   // s_p staged / the previous half's conv1_2 steps are done with s_x
    // ---- conv1_1 channels [32 hf, 32 hf + 32) on the halo, activated and split, into s_x
    for (int g = wave; g < HG; g += NT / 64) {
      const int hp = g * 32 + l32;
      const int hy = hp / HWD, hx = hp - hy * HWD;
      const int y = y0 - 1 + hy, x = x0 - 1 + hx;
      const bool inimg = hp < HPX && y >= 0 && y < a.H && x >= 0 && x < a.W;
      // the pixel's 3 x 3 input neighbourhood (channels 0-2 of each 32-byte chunk) from the staged
      // region (out-of-image halo pixels are zeroed below); then K slot j of lane half h in K step
      // kk is k = 16 kk + 8 h + j = 9 ky + 3 kx + c (conv_x3_rgb's packing)
      f32x4 nb[9];
      const int ry = min(hy, HH - 1), rx = hx;   // (groups past the halo read a valid slot)
#pragma unroll
      for (int t = 0; t < 9; ++t) nb[t] = s_in[ry + t / 3][rx + t % 3];
      auto kval = [&](int k) __attribute__((always_inline)) { return k < 27 ? nb[k / 3][k % 3] : 0.f; };
      f32x16 acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        f32x4 v0, v1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = h ? kval(16 * kk + 8 + j) : kval(16 * kk + j);
          if (j < 4) v0[j] = v;
          else v1[j - 4] = v;
        }
        f16x4 h0, l0, h1, l1;
        split4(v0, h0, l0);
        split4(v1, h1, l1);
        const f16x8 Bh = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        const f16x8 Bl = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        const f16x8 A0 = a.w1[((kk * 2 + 0) * 2 + h) * 64 + 32 * hf + l32];
        const f16x8 A1 = a.w1[((kk * 2 + 1) * 2 + h) * 64 + 32 * hf + l32];
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, Bh, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, Bl, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, Bh, acc1, 0, 0, 0);
      }
      // register r: channel 32 hf + (r & 3) + 8 (r >> 2) + 4 h of halo pixel hp; registers
      // 4c .. 4c + 3 are elements 4h .. 4h + 3 of chunk c of the half
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 32 * hf + 8 * c + 4 * h + e;
          float t = acc1[4 * c + e] * a.s1_inv + s_p[co];
          t = act_f<RR>(t, a.act1, s_p[128 + co]);
          bad |= inimg && !(__builtin_fabsf(t) < 65504.f);
          v[e] = inimg ? t : 0.f;
        }
        f16x4 hi, lo;
        split4(v, hi, lo);
        *(f16x4*)((_Float16*)&s_x[0][c][hp] + 4 * h) = hi;
        *(f16x4*)((_Float16*)&s_x[1][c][hp] + 4 * h) = lo;
      }
    }
    __syncthreads();
    // ---- conv1_2 pairs 2 hf, 2 hf + 1 (6 steps of (pair, ky)) from the resident halo
    for (int i = 0; i < 6; ++i) {
      const int st = 6 * hf + i, b = st & 1;
      if (st + 1 < 12) load_w(st + 1);
      const int pp = i / 3, ky = i - 3 * pp;
      const f16x8* sw = &s_w[b][h * 64 + l32];
      const f16x8* sx = &s_x[0][2 * pp + h][(wave + ky) * HWD + l32];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        f16x8 A[2][2], B[2];
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
#pragma unroll
          for (int wm = 0; wm < 2; ++wm) A[wm][hl] = sw[(kx * 2 + hl) * 2 * 64 + wm * 32];
          B[hl] = sx[hl * 4 * HPS + kx];
        }
#pragma unroll
        for (int wm = 0; wm < 2; ++wm) {
          acc2[wm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[0], acc2[wm], 0, 0, 0);
          acc2[wm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[1], acc2[wm], 0, 0, 0);
          acc2[wm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][1], B[0], acc2[wm], 0, 0, 0);
        }
      }
      if (st + 1 < 12) store_w(b ^ 1);   // buffer b ^ 1 was last read in the previous step
      __syncthreads();   // the next slab is in LDS; this one may be overwritten
    }
  }
  // ---- conv1_2's epilogue with the pool (model.py:29 pool1_stage1, 2 x 2 / 2): the pair max of
  // neighbouring columns by a DPP swap (conv_x3_f16 hpool); pool2: the row pair's max too (rows
  // y, y + 1 are waves 2i, 2i + 1: the odd wave hands its pair maxima over in LDS) and the pooled
  // value stored into the padded pooled buffer, so conv2_1 reads a plain input (no row-pair max
  // in its staging).  max is exact in any order: the bits of maxpool2 / vpool2.
  const int y = y0 + wave, x = x0 + l32;
  const bool ok = y < a.H && x < a.W;
  float* out_f = a.out + (size_t)n * a.out_fs;
  f32x4 pv[2][4];
#pragma unroll
  for (int wm = 0; wm < 2; ++wm)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int co = wm * 32 + 8 * q + 4 * h;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc2[wm][4 * q + e] * a.s2_inv + s_p[64 + co + e];
        t = act_f<RR>(t, a.act2, s_p[192 + co + e]);
        bad |= ok && !(__builtin_fabsf(t) < 65504.f);
        v[e] = t;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = fmaxf(v[e], __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[e]), 0xB1, 0xF, 0xF, false)));
      pv[wm][q] = v;
    }
  if (!a.pool2) {
#pragma unroll
    for (int wm = 0; wm < 2; ++wm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = wm * 32 + 8 * q + 4 * h;
        if (ok && !(x & 1))
          *(f32x4*)(out_f + (size_t)(co >> 3) * a.out_chs + ((size_t)y * (a.W / 2) + (x >> 1)) * 8 + (co & 7)) = pv[wm][q];
      }
  } else {
    // the K loop ended on a barrier: s_x is free.  Slot (row pair, wm, q, h, even lane / 2).
    f32x4* xch = reinterpret_cast<f32x4*>(&s_x[0][0][0]);
    auto slot = [&](int wm, int q) { return (((wave >> 1) * 8 + wm * 4 + q) * 2 + h) * 16 + (l32 >> 1); };
    if (wave & 1) {
#pragma unroll
      for (int wm = 0; wm < 2; ++wm)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (!(l32 & 1)) xch[slot(wm, q)] = pv[wm][q];
    }
    __syncthreads();
    if (!(wave & 1) && ok && y + 1 < a.H && !(x & 1)) {
      float* op = out_f + ((size_t)((y >> 1) + a.out_pad) * a.out_wp + (x >> 1) + a.out_pad) * 8;
#pragma unroll
      for (int wm = 0; wm < 2; ++wm)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co = wm * 32 + 8 * q + 4 * h;
          const f32x4 u = xch[slot(wm, q)];
          f32x4 v = pv[wm][q];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], u[e]);
          *(f32x4*)(op + (size_t)(co >> 3) * a.out_chs + (co & 7)) = v;
        }
    }
  }
  if (bad) atomicOr(a.range_flag, 1);
}

}  // namespace

bool x3_c12_fits(const ConvLaunch& l1, const ConvLaunch& l2) {
  // hpool 1: the pair-max buffer (out_pad 0); 2: the pooled buffer, any pad ring
  return l1.ks == 3 && l1.cin_chunks == 1 && l1.cout == 64 && l1.in_pad >= 1 && l1.in_coff == 0 &&
         l2.ks == 3 && l2.cin_chunks == 8 && l2.cout == 64 && l2.bco == 64 && (l2.hpool == 1 || l2.hpool == 2) &&
         !(l2.W & 1) && l1.H == l2.H && l1.W == l2.W && l1.n == l2.n && l2.out_coff == 0 &&
         (l2.hpool == 2 ? l2.out_pad >= 0 : l2.out_pad == 0) && (l2.out_cs & 7) == 0 && l2.out_cs >= 64 && l1.wx3 &&
         l2.wx3 && l1.range_flag;
}

hipError_t launch_conv_x3_c12(const ConvLaunch& l1, const ConvLaunch& l2, hipStream_t s) {
  if (!x3_c12_fits(l1, l2)) {
    set_error("conv_x3_c12: needs conv1_1 (3 -> 64, rgb-packed) and conv1_2 (64 -> 64, 64-channel tile, pair-max output)");
    return hipErrorInvalidValue;
  }
  C12Args a{};
  const long long in_chs = (long long)(l1.H + 2 * l1.in_pad) * (l1.W + 2 * l1.in_pad) * 8;
  a.in = l1.in;
  a.in_fs = in_chs * (l1.in_cs / 8);
  a.in_pad = l1.in_pad;
  a.w1 = (const f16x8*)l1.wx3;
  a.b1 = l1.bias; a.sl1 = l1.slope; a.s1_inv = l1.wscale_inv; a.act1 = l1.act;
  a.w2 = (const f16x8*)l2.wx3;
  a.b2 = l2.bias; a.sl2 = l2.slope; a.s2_inv = l2.wscale_inv; a.act2 = l2.act;
  a.out = l2.out;
  a.pool2 = l2.hpool == 2;
  a.out_pad = a.pool2 ? l2.out_pad : 0;
  a.out_wp = l2.W / 2 + 2 * a.out_pad;
  a.out_chs = a.pool2 ? (long long)(l2.H / 2 + 2 * a.out_pad) * a.out_wp * 8 : (long long)l2.H * (l2.W / 2) * 8;
  a.out_fs = a.out_chs * (l2.out_cs / 8);
  a.H = l1.H; a.W = l1.W;
  a.tiles_x = (l1.W + TW - 1) / TW;
  a.tiles_y = (l1.H + TH - 1) / TH;
  a.range_flag = l1.range_flag;
  const long long nb = (long long)l1.n * a.tiles_x * a.tiles_y;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("conv_x3_c12: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  if (a.act1 == ACT_RELU && a.act2 == ACT_RELU) hipLaunchKernelGGL(conv_x3_c12<true>, dim3(a.nblocks), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(conv_x3_c12<false>, dim3(a.nblocks), dim3(NT), 0, s, a);
  return hipGetLastError();
}

double conv_x3_c12_mfma_flops(const ConvLaunch& l1) {
  const double tiles = (double)l1.n * ((l1.W + TW - 1) / TW) * ((l1.H + TH - 1) / TH);
  return tiles * 3.0 * 2.0 * (64.0 * 32.0 * HPS + 64.0 * 64.0 * 9.0 * TH * TW);
}

}  // namespace isl
