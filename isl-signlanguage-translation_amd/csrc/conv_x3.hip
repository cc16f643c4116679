// Direct convolution (3x3 / 1x1 / 7x7, stride 1, "same" padding) on the gfx950
// FP16 matrix cores with fp32 accuracy: every fp32 operand is split into two
// fp16 halves, x = x_hi + x_lo, and each product is taken as
//     x*w ~= x_hi*w_hi + x_hi*w_lo + x_lo*w_hi          (3 x v_mfma_f32_32x32x16_f16)
// with fp32 accumulation.  The dropped x_lo*w_lo term and the split residuals
// are ~2^-21 relative per product, i.e. fp32 round-off territory: on body_25
// the max-normalised error vs fp64 is 2.2e-6 / 3.9e-6 (PAF / heat), the same as
// native fp32 (2.2e-6 / 3.7e-6), against north_star's 1e-4 bar.  Three fp16
// MFMAs cost 3/16 of one FP32 MFMA of the same K, so the convolutions run at
// up to 16/3 = 5.3x the FP32 matrix peak.
//
// Replaces every nn.Conv2d (+ReLU / PReLU) of src/model.py:25-64 (make_layers,
// make_layers_Mconv).
//
// Range: weights are scaled by a per-layer power of two 2^s (host, exact) so
// that max|w| sits in [2^13, 2^14): the lo halves stay normal fp16 numbers, and
// the epilogue multiplies by 2^-s (exact).  Activations are split unscaled;
// their lo halves may be fp16 subnormals, an absolute error <= 2^-25 that is
// negligible against the tensor maxima the tolerance is normalised by.  An
// activation with |x| >= 65504 would not split: every epilogue checks its
// outputs and raises the net's range flag (isl_net_check / ISL_E_RANGE), and
// the host then re-runs on the fp32 kernels.
//
// GEMM view (same tiling as conv.hip):  D[co][px] = sum_k W[co][k] X[k][px],
// k = (ky, kx, ci).  One MFMA K-step = one tap (ky, kx) x 16 input channels =
// two 8-channel chunks of the NC8HW8 buffer; lane half h (= lane >> 5) carries
// chunk h of the pair, 8 channels = one 16-byte fp16 fragment.
//   A (32 rows)  = 32 output channels     lane: co = l & 31, k = 8h + j
//   B (32 cols)  = 32 output pixels       lane: px = l & 31, k = 8h + j
//   D            = lane holds pixel l&31, channels (r&3)+8(r>>2)+4(l>>5)
//
// K loop: one step = (chunk pair, kernel row ky).
//   weights: the pre-split slab [kx][hi|lo][h][BCO] x 16 B arrives by LDS-DMA
//            (global_load_lds_dwordx4, lane-linear, no VGPRs);
//   input:   the row segment of the flattened pixel tile (one contiguous run of
//            the padded buffer, see conv.hip) is loaded as fp32, split into
//            fp16 hi / lo in registers and written as [hi|lo][h][px] x 16 B.
// Double-buffered, one barrier per step; per step and wave KS taps x WM*WN
// accumulator tiles x 3 MFMAs.
//
// Variants (template VAR bits):
//   512   row union (3x3 on 512-pixel tiles): the three kernel rows of a chunk pair
//         are staged once as one run, a third per ky step, by loader waves, while
//         DMA waves stream the weights (role split, see the union loop);
//   1024  canonical K ranges (in-block): the chunk pairs are summed in S ranges, each from
//         zero; the first h = ceil(S / 2) range sums are added in order, the others in order,
//         then the two halves (x3_canonical_order) -- the same bits as 2048;
//   2048  split-K across blocks: each block writes one range's sum, x3_splitk_reduce
//         adds them in range order.  S depends on the layer shape only
//         (x3_canonical_ranges), so a frame gives the same bits at any batch size
//         whether its ranges ran in one block (large grids) or across blocks (small
//         grids: batch-1 frames).
//   4096  two chunk pairs per K step (1x1 layers on 256-channel tiles, x3_wide1);
//   16384 development only: s_memtime stamps of the union loop (tools/convbench;
//         compiled only with -DISLPOSE_DEV, never into libislpose.so).
//   32768 pooled input (ConvLaunch::vin): the input is the pair-max buffer of the 2x2
//         pool before this layer; staging takes the row-pair max (x3_vin_ok).
//   131072 the row union on v_mfma_f32_16x16x32_f16 (products folded into K, x3_m16;
//         development build only).
//   32    two K groups per block (with 1024): waves [0, NW) sum the first half of the K ranges,
//         waves [NW, 2 NW) the second half, each group on its own double buffers, one barrier
//         per step for both; the halves meet in LDS at the end (small grids: one block per CU
//         with twice the waves, so one group's step latency overlaps the other's MFMAs);
//   16    the 1x1 pair Mconv6 -> Mconv7 in one launch (ConvLaunch::cout7): the block holds
//         every Mconv6 output channel of its pixel tile in registers, turns the activated
//         values into the split B operand of Mconv7 in place (the MFMA D layout of a 32-row
//         tile is two K=16 B fragments once Mconv7's K is packed in that order, pack_x3_f7),
//         each wave sums its 64 channels' Mconv7 products, and the waves' sums are added in
//         wave order through LDS.  The Mconv6 output never goes to HBM.
// conv_x3_rgb: the 3-channel first layers (conv1_1) with K packed as the 27 real
// (ky, kx, c) values instead of 9 taps x 16 channels.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "internal.h"

namespace isl {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct X3Args {
  const float* in;
  float* out;
  const f16x8* wpk;
  const float* bias;
  const float* slope;
  int* range_flag;
  long long in_fs, in_chs;      // frame / chunk strides (floats) of the input buffer
  long long out_fs, out_chs;
  float wscale_inv;             // 2^-s
  int in_pad, out_pad;
  int H, W, cin_chunks, pairs, cout, co_tiles, px_tiles, tpx, act, nblocks;
  int ksplit;                   // K ranges (VAR 1024 / 2048)
  int nfr;                      // frames (split-K partial-sum layout)
  float* ws;                    // split-K partial sums [ksplit][nfr][cout/8][H*W][8]
  unsigned long long* dbg;      // VAR 16384 (development): s_memtime stamps of block 0
  int hpool;                    // ConvLaunch::hpool: out is the [n][chunk][H][W/2][8] pair-max buffer
  int vin;                      // ConvLaunch::vin: in is the [n][chunk][2H][W][8] pair-max buffer of a pool
  const X3Fold* fold;           // VAR 8192: per input chunk, the split-K partials it is folded from
  int abl;                      // development (-DISLPOSE_DEV, ISLPOSE_X3_ABL): generic-loop ablations
  // VAR 16 (the fused 1x1 pair): Mconv7's filters in the fused K order (pack_x3_f7), bias,
  // PReLU slopes, activation, 2^-s and output channels; out / out_* describe Mconv7's output
  const f16x8* wpk7;
  const float* bias7;
  const float* slope7;
  float wscale7_inv;
  int cout7, act7;
  int bco_pack;                 // conv_x3_wr: output channels per tile of the weight packing (c.bco)
  // tail tiles (x3_tail_plan): blocks [0, nb_full) take each frame's first full_tiles tiles of tpx
  // pixels, blocks [nb_full, nblocks) the frame's rest in tail_tiles tiles of ttpx pixels (0: one
  // tiling of px_tiles tiles)
  int nb_full, full_tiles, tail_tiles, ttpx;
};

// u / d for 0 <= u < 2^20, d >= 1, through the fp32 reciprocal r = 1/d: (u + 0.5) / d sits
// >= 0.5 / d away from an integer, and (u + 0.5) * r (two roundings, relative error < 2^-23)
// is off by < 2^20 / d * 2^-23 = 0.125 / d, so the truncation is exact
__device__ __forceinline__ int x3_div(int u, float r) { return (int)(((float)u + 0.5f) * r); }

// VIN: the staged input pixel at padded position (yy, xx) of chunk plane `src` (the pair-max
// buffer [2H][W][8] of the pool this layer reads): max of rows 2(yy-pad), 2(yy-pad)+1,
// zero on the ring -- the values maxpool2_kernel / vpool2_kernel would have stored
__device__ __forceinline__ void x3_vin_load(const float* src, int yy, int xx, const X3Args& a, float4& lo4,
                                            float4& hi4) {
  const int y = yy - a.in_pad, x = xx - a.in_pad;
  if (y < 0 || y >= a.H || x < 0 || x >= a.W) {
    lo4 = hi4 = float4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const float* p0 = src + ((size_t)(2 * y) * a.W + x) * 8;
  const float* p1 = p0 + (size_t)a.W * 8;
  const float4 a0 = *(const float4*)p0, a1 = *(const float4*)(p0 + 4);
  const float4 b0 = *(const float4*)p1, b1 = *(const float4*)(p1 + 4);
  lo4 = float4{fmaxf(a0.x, b0.x), fmaxf(a0.y, b0.y), fmaxf(a0.z, b0.z), fmaxf(a0.w, b0.w)};
  hi4 = float4{fmaxf(a1.x, b1.x), fmaxf(a1.y, b1.y), fmaxf(a1.z, b1.z), fmaxf(a1.w, b1.w)};
}

// x = hi + lo for 8 fp32 values: packed RNE conversions (v_cvt_pk_f16_f32), hi converted
// back once for the residual -- the same bits as hi = (f16)x; lo = (f16)(x - (f32)hi)
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void x3_split8(const f32x4& a, const f32x4& b, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x = k < 2 ? f32x2{a[2 * k], a[2 * k + 1]} : f32x2{b[2 * k - 4], b[2 * k - 3]};
    const f16x2 h = __builtin_convertvector(x, f16x2);
    const f32x2 hf = __builtin_convertvector(h, f32x2);
    // two scalar subtractions: hipcc would pack them into v_pk_add_f32, which beside the
    // other waves' MFMAs measured 0.6 % slower (tools/archive/gpu_split_ab.sh, profiles/r02/split_ab/)
    f32x2 r;
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r.x) : "v"(x.x), "v"(hf.x));
    asm volatile("v_sub_f32 %0, %1, %2" : "=v"(r.y) : "v"(x.y), "v"(hf.y));
    const f16x2 l = __builtin_convertvector(r, f16x2);
    hi[2 * k] = h.x; hi[2 * k + 1] = h.y;
    lo[2 * k] = l.x; lo[2 * k + 1] = l.y;
  }
}

// Split-K reduction: the ranges' sums added in range order (the order of the in-block
// ranges, so both give the same bits), then the epilogue of conv_x3_f16 (x 2^-s,
// bias, activation, range check, masked stores).  One thread per (frame, chunk, pixel,
// 4-channel half): neighbouring lanes read the two halves of a pixel's 32-byte chunk, so a
// wave's loads and stores are contiguous.  The ranges' loads are all issued before the first
// add (up to 8 in flight; the batch-1 frames' reduces had waited on one range at a time:
// 5.0 us per launch at 23x41).
// x3_canonical_order: ranges [0, h) summed in order, ranges [h, S) in order, then the two
// halves, h = ceil(S / 2) -- the order of the in-block ranges (one or two K groups)
template <int S>
__device__ __forceinline__ f32x4 x3_sum_ranges(const float* p, size_t stride) {
  f32x4 part[S];
#pragma unroll
  for (int k = 0; k < S; ++k) part[k] = __builtin_nontemporal_load((const f32x4*)(p + k * stride));
  constexpr int H = (S + 1) / 2;
  f32x4 lo = f32x4{0.f, 0.f, 0.f, 0.f}, hi = lo;   // onto +0, as the in-block sums
#pragma unroll
  for (int k = 0; k < H; ++k) lo += part[k];
  if constexpr (S > H) {
#pragma unroll
    for (int k = H; k < S; ++k) hi += part[k];
    return lo + hi;
  }
  return lo;
}

// one (frame n, chunk cc, pixel m, 4-channel half h) of the reduction
__device__ __forceinline__ void x3_reduce_item(const X3Args& a, int n, int cc, int m, int h) {
  const int HW = a.H * a.W, c8 = (a.cout + 7) / 8;
  const int co = 8 * cc + 4 * h;
  if (co >= a.cout) return;
  const size_t plane = (size_t)HW * 8;
  const float* p = a.ws + ((size_t)n * c8 + cc) * plane + (size_t)m * 8 + 4 * h;
  const size_t split_stride = (size_t)a.nfr * c8 * plane;
  // the epilogue's operands requested with the partials, not one round trip after them
  const f32x4 b = *(const f32x4*)(a.bias + co);
  const f32x4 sl = a.act == ACT_PRELU ? *(const f32x4*)(a.slope + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 sum;
  switch (a.ksplit) {   // uniform: one straight-line body per range count (loads in flight together)
    case 2: sum = x3_sum_ranges<2>(p, split_stride); break;
    case 3: sum = x3_sum_ranges<3>(p, split_stride); break;
    case 4: sum = x3_sum_ranges<4>(p, split_stride); break;
    case 5: sum = x3_sum_ranges<5>(p, split_stride); break;
    case 6: sum = x3_sum_ranges<6>(p, split_stride); break;
    case 7: sum = x3_sum_ranges<7>(p, split_stride); break;
    case 8: sum = x3_sum_ranges<8>(p, split_stride); break;
    default: {
      const int hh = (a.ksplit + 1) / 2;
      f32x4 hi = f32x4{0.f, 0.f, 0.f, 0.f};
      sum = hi;
      for (int k = 0; k < hh; ++k) sum += *(const f32x4*)(p + k * split_stride);
      for (int k = hh; k < a.ksplit; ++k) hi += *(const f32x4*)(p + k * split_stride);
      if (a.ksplit > hh) sum += hi;
    }
  }
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = sum[e] * a.wscale_inv + b[e];
  if (a.act == ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
  } else if (a.act == ACT_PRELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
  }
  bool bad = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) bad |= co + e < a.cout && !(__builtin_fabsf(v[e]) < 65504.f);
  const int y = m / a.W, x = m - y * a.W, Wo = a.W + 2 * a.out_pad;
  float* oc = a.out + (size_t)n * a.out_fs + (size_t)cc * a.out_chs +
              (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8 + 4 * h;
  if (co + 3 < a.cout) {
    *(f32x4*)oc = v;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (co + e < a.cout) oc[e] = v[e];
  }
  if (bad) atomicOr(a.range_flag, 1);
}

// input segment capacity in pixels for a BPX-pixel tile (host: tile_pixels)
constexpr int x3_segmax(int bpx) { return bpx + 64; }
// capacity of the row-union run (VAR 512): 2 x (1536 + 4 x 857) x 16 B = 155 KiB of LDS
// with the 128-channel 3x3 weight slabs
constexpr int x3_segu_max() { return 856; }

template <int KS, int WAVES_M, int WAVES_N, int WM, int WN, int VAR, int OCC>
__global__ void __launch_bounds__(WAVES_M * WAVES_N * 64 * ((VAR & 32) ? 2 : 1), OCC) conv_x3_f16(X3Args a) {
  // VAR 32: two K groups of WAVES_M x WAVES_N waves each (see the generic loop)
  constexpr bool G2 = (VAR & 32) != 0;
  constexpr int NG = G2 ? 2 : 1;
  constexpr int NWAVES = WAVES_M * WAVES_N;      // waves per K group
  constexpr int NTG = NWAVES * 64;               // threads per K group
  constexpr int NT = NG * NTG;
  constexpr int BCO = WAVES_M * WM * 32;
  constexpr int BPX = WAVES_N * WN * 32;
  constexpr int P = KS / 2;
  constexpr int SEGMAX = x3_segmax(BPX);
  // VAR 4096 (1x1 layers, 256-channel tiles): two chunk pairs per K step
  constexpr int PPS = (VAR & 4096) ? 2 : 1;
  static_assert(PPS == 1 || KS <= 3, "two pairs per step: 1x1 / 3x3 layers");
  constexpr int WSLAB1 = KS * 2 * 2 * BCO;       // one pair: [kx][hi|lo][h][BCO]
  constexpr int WSLAB = PPS * WSLAB1;            // 16-byte units per step
  constexpr int SEGP = SEGMAX + 1;               // + one dummy slot idle staging items write to
  constexpr int XSLAB = 2 * 2 * PPS * SEGP;      // 16-byte units: [hi|lo][chunk of the step][px]
  constexpr int BUF = WSLAB + XSLAB;
  constexpr int IT = (2 * PPS * SEGMAX + NTG - 1) / NTG; // staging items (chunk, px) per thread of a group
  static_assert(WSLAB % 64 == 0, "weight slab is whole 1 KiB DMA pieces");
  static_assert(BPX <= SEGMAX, "segment must hold a tile");
  constexpr bool UNION = (VAR & 512) != 0;
  // VAR 131072: the row-union loop on v_mfma_f32_16x16x32_f16 (see the M16 loop below)
  constexpr bool M16 = (VAR & 131072) != 0;
  static_assert(!M16 || (UNION && KS == 3 && WAVES_M == 2 && WAVES_N == 8 && WM == 2 && WN == 2),
                "16x16x32 form: the 128-channel row-union block (16 waves of 64co x 64px)");
  // VAR 65536: one input buffer (two barriers per step) so that a wider pixel tile fits
  // beside the double-buffered weight slabs (7x7 on 384 pixels: the 56 KiB slab per step
  // is amortised over 1.5x the pixels)
  constexpr bool SIB = (VAR & 65536) != 0;
  constexpr int SEGUP = x3_segu_max() + 1;       // + dummy slot
  constexpr int XSLABU = 2 * 2 * SEGUP;          // [hi|lo][h][px]
  constexpr int SMEM0 = UNION ? 2 * WSLAB + 2 * XSLABU : SIB ? 2 * WSLAB + XSLAB
                      : (VAR & 128) ? 3 * WSLAB + 2 * XSLAB : NG * 2 * BUF;
  static_assert(!(SIB && UNION), "one input buffer: generic loop only");
  // VAR 16: Mconv6 -> Mconv7 fused (the epilogue below); its LDS: the epilogue parameters and
  // the waves' Mconv7 sums of one pass (WAVES_N pixel tiles), [WAVES_M][WAVES_N * 32][F7_ROWS]
  constexpr bool FUSE67 = (VAR & 16) != 0;
  constexpr int F7_ROWS = 68;                    // 64 rows + 4 (staggers the banks of the pixel rows)
  constexpr int F7_SMEM = FUSE67 ? ((2 * BCO + 128) * 4 + WAVES_M * WAVES_N * 32 * F7_ROWS * 4 + 15) / 16 : 0;
  constexpr int SMEM = SMEM0 > F7_SMEM ? SMEM0 : F7_SMEM;
  static_assert(SMEM * 16 <= 160 * 1024, "LDS");
  constexpr bool RANGED = (VAR & 1024) != 0;
  constexpr bool SPLIT = (VAR & 2048) != 0;
  constexpr bool STAMP = (VAR & 16384) != 0;
  constexpr bool VIN = (VAR & 32768) != 0;      // ConvLaunch::vin (pooled-input staging)
  // VAR 8192: input chunks whose producer left split-K partial sums (ConvLaunch::fold) are
  // staged as the reduction x3_splitk_reduce would have stored them
  constexpr bool FOLD = (VAR & 8192) != 0;
  // VAR 256: a 64-channel block of weights packed for 128-channel tiles (small grids: two
  // independent blocks per 128-channel tile, so one block's step latency overlaps the
  // other's MFMAs); its slab rows are the halves of the packed 128-channel rows
  constexpr bool HALFCO = (VAR & 256) != 0;
  static_assert(!HALFCO || (BCO == 64 && !UNION && !M16 && PPS == 1), "half-tile blocks: generic loop, 64 channels");
  // VAR 128: the generic loop with weights and inputs prefetched two K steps ahead (three
  // weight buffers, two register slots), a raw s_barrier with counted vmcnt waits instead of
  // __syncthreads (which drains every LDS-DMA in flight): small grids, whose short steps
  // otherwise wait out one L2 round trip each
  constexpr bool DEEP = (VAR & 128) != 0;
  static_assert(!DEEP || (!UNION && !M16 && !SIB && !FOLD && !VIN && !(VAR & 16384)), "deep prefetch: plain generic loop");
  static_assert(!(FOLD && (VIN || UNION || M16 || KS > 3 || PPS > 1)), "fold: the generic loop of 1x1 / 3x3 layers");
  static_assert(!(UNION && (RANGED || SPLIT)), "K ranges run on the generic loop");
  static_assert(PPS == 1 || !(UNION || M16 || HALFCO || DEEP || FOLD || VIN), "two pairs per step: generic loop");
  static_assert(!G2 || (RANGED && !SPLIT && !UNION && !M16 && !SIB && !DEEP && !FOLD && !VIN && !HALFCO && PPS == 1 &&
                        !FUSE67 && !STAMP),
                "two K groups: in-block K ranges on the plain generic loop");
  __shared__ f16x8 smem[SMEM];

  // XCD-aware tile order (conv.hip): co-tiles of a pixel tile, then neighbouring
  // pixel tiles, on one XCD / L2.
  int bid = blockIdx.x;
  // tail tiles: the full tiles' blocks are dispatched first (whole rounds of one block per CU),
  // then the tails', each class spread over the XCDs on its own
  const bool tail = a.nb_full > 0 && bid >= a.nb_full;
  {
    const int b0 = tail ? a.nb_full : 0;
    const int nb = a.nb_full > 0 ? (tail ? a.nblocks - a.nb_full : a.nb_full) : a.nblocks;
    const int lb = bid - b0, q = nb >> 3, r = nb & 7, xcd = lb & 7, k = lb >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  int ks_i = 0;
  if constexpr (SPLIT) {
    ks_i = bid % a.ksplit;
    bid /= a.ksplit;
  }
  const int co_t = bid % a.co_tiles;
  const int rest = bid / a.co_tiles;
  const int ntile = tail ? a.tail_tiles : a.nb_full > 0 ? a.full_tiles : a.px_tiles;
  const int pt = rest % ntile;
  const int n = rest / ntile;

  const int HW = a.H * a.W;
  const int m0 = tail ? a.full_tiles * a.tpx + pt * a.ttpx : pt * a.tpx;   // tpx = BPX unless the image is very narrow
  const int mlast = min(m0 + (tail ? a.ttpx : a.tpx), HW) - 1;
  const int Wi = a.W + 2 * a.in_pad;
  const float inv_wi = 1.f / (float)Wi;          // VIN: x3_div
  const int ya = m0 / a.W, xa = m0 - ya * a.W;
  const int yb = mlast / a.W, xb = mlast - yb * a.W;
  const int La = (ya + a.in_pad) * Wi + xa + a.in_pad;
  const int Lb = (yb + a.in_pad) * Wi + xb + a.in_pad;
  const int seg = Lb - La + 2 * P + 1;
  const float* in_f = a.in + (size_t)n * a.in_fs;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = G2 ? __builtin_amdgcn_readfirstlane(wave / NWAVES) : 0;   // K group (VAR 32)
  const int wave_g = wave - grp * NWAVES, tid_g = tid - grp * NTG;           // within the group
  const int wave_m = wave_g % WAVES_M, wave_n = wave_g / WAVES_M;
  const int h = lane >> 5, l32 = lane & 31;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave_g);

  int rel[WN];
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int j = (wave_n * WN + wn) * 32 + l32;
    const int m = min(m0 + j, mlast);
    const int y = m / a.W, x = m - y * a.W;
    rel[wn] = (y + a.in_pad) * Wi + x + a.in_pad - La;
  }

  const int T = a.pairs / PPS * KS;              // K steps (PPS == 2: the host checks pairs is even)

  f32x16 acc[WM][WN];
#pragma unroll
  for (int wm = 0; wm < WM; ++wm)
#pragma unroll
    for (int wn = 0; wn < WN; ++wn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[wm][wn][r] = 0.f;

  // one tap (kx) of a K step: WM x WN accumulator tiles x 3 MFMAs from the weight
  // slab sw and the input run sx (both already offset to this lane's fragments)
  // big tiles (the tail-tile families): a wave whose pixel granules all lie past the tile (tail and
  // last tiles) skips its MFMAs -- the live waves of a tile of 128 k pixels stay spread evenly over
  // the SIMDs.  (The 128-pixel family keeps its loops branch-free.)
  constexpr bool SKIP_DEAD = BPX >= 256 && !FUSE67 && !M16;
  const bool wave_live = !SKIP_DEAD || m0 + (wave_u / WAVES_M) * WN * 32 <= mlast;   // (uniform)
  auto tap = [&](const f16x8* sw, const f16x8* sx, int sx_plane, int kx) __attribute__((always_inline)) {
    if (SKIP_DEAD && !wave_live) return;
    f16x8 A[WM][2], B[WN][2];
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) A[wm][hl] = sw[(kx * 2 + hl) * 2 * BCO + wm * 32];
#pragma unroll
      for (int wn = 0; wn < WN; ++wn) B[wn][hl] = sx[hl * 2 * sx_plane + rel[wn] + kx];
    }
#pragma unroll
    for (int wm = 0; wm < WM; ++wm)
#pragma unroll
      for (int wn = 0; wn < WN; ++wn) {
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[wn][0], acc[wm][wn], 0, 0, 0);
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[wn][1], acc[wm][wn], 0, 0, 0);
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][1], B[wn][0], acc[wm][wn], 0, 0, 0);
      }
  };

  if constexpr (M16) {
    // Row union on v_mfma_f32_16x16x32_f16, two taps per K step.
    // Per 16x16 (co x px) block a lane carries K group g = lane >> 4 (8 fp16 values of
    // chunk g & 1 of the pair).  The three products of a tap fold into K:
    //   M(tap):   [Ahi c0 | Ahi c1 | Alo c0 | Alo c1] x [Bhi c0 | Bhi c1 | Bhi c0 | Bhi c1]
    //             = x_hi w_hi + x_hi w_lo of the tap, every K lane used;
    //   X(a, b):  [Ahi c0 @a | Ahi c1 @a | Ahi c0 @b | Ahi c1 @b] x [Blo c0 @a | .. | Blo c1 @b]
    //             = the x_lo w_hi terms of two taps.
    // A K step is two consecutive taps of the (pair, ky, kx) sequence -- M, M, X: 48 MFMAs
    // per wave, none padded (a step of one kernel row has 3 taps, i.e. half an X left
    // over).  Pairs come in twos (host: even pair count) so the 9 taps of a pair pair up
    // across the pair boundary: in every 9 steps, step 4 reads pair 2k's last tap and pair
    // 2k+1's first, each from its own union run.  Weights: the packed [pair][ky][kx][hi|lo]
    // [h][BCO] array in tap order, 16 KiB per step by LDS-DMA (DMA waves 10-15, one step
    // ahead).  Input: the 3-row union run of a pair, double-buffered; loader waves 0-9
    // stage the next pair a quarter per step (steps 0-3 of a 9-step cycle pair 2k+1, steps
    // 5-8 pair 2k+2), stored at the step end, so a run is complete before the first step
    // that reads it and is overwritten only after the last step that read it has passed
    // its barrier.  Same sums as the 32x32x16 loop up to the fp32 accumulation order.
    static_assert(NWAVES == 16, "role split sized for 16-wave blocks");
    constexpr int LOADER_WAVES = 10, DMA_WAVES = NWAVES - LOADER_WAVES;
    constexpr int WS2 = 2 * 4 * BCO;                            // one step: 2 taps x [hi|lo][h][BCO]
    constexpr int NP = WS2 / 64;
    constexpr int DPW = (NP + DMA_WAVES - 1) / DMA_WAVES;
    constexpr int SEGUP = (x3_segu_max() + 1 + 15) / 16 * 16;   // plane stride: a multiple of 256 B
    constexpr int XSLABU = 2 * 2 * SEGUP;                       // [hi|lo][h][px]
    static_assert((2 * WS2 + 2 * XSLABU) * 16 <= 160 * 1024, "LDS");
    const bool loader = wave_u < LOADER_WAVES;
    const int Pw = P * Wi;
    const int segu = Lb - La + 2 * Pw + 2 * P + 1;
    const long long ubase = (long long)La - Pw - P;
    const int quarter = (2 * segu + 3) / 4;                     // staging items per step (<= 428)
    // staging item of this thread in quarter q (q uniform, run-time): chunk of the pair
    // ih, pixel of the run px (-1: idle)
    auto item = [&](int q, int& ih, int& px) __attribute__((always_inline)) {
      const int it = q * quarter + tid;
      const bool ok = tid < quarter && it < 2 * segu;
      ih = ok && it >= segu ? 1 : 0;
      px = ok ? it - ih * segu : -1;
    };
    f32x4 ru[2];
    auto load_q = [&](int c2, int q) __attribute__((always_inline)) {
      int ih, px;
      item(q, ih, px);
      if (px >= 0) {
        const int c = min(2 * c2 + ih, a.cin_chunks - 1);
        if constexpr (VIN) {
          const int u = (int)ubase + px, yy = x3_div(u, inv_wi);
          float4 l4, h4;
          x3_vin_load(in_f + (size_t)c * a.in_chs, yy, u - yy * Wi, a, l4, h4);
          ru[0] = f32x4{l4.x, l4.y, l4.z, l4.w};
          ru[1] = f32x4{h4.x, h4.y, h4.z, h4.w};
        } else {
          const float* src = in_f + (size_t)c * a.in_chs + (size_t)(ubase + px) * 8;
          ru[0] = *(const f32x4*)src;
          ru[1] = *(const f32x4*)(src + 4);
        }
      }
    };
    auto store_q = [&](int q, int bx) __attribute__((always_inline)) {
      int ih, px;
      item(q, ih, px);
      f16x8* sx = smem + 2 * WS2 + bx * XSLABU;
      f16x8 hi, lo;
      x3_split8(ru[0], ru[1], hi, lo);
      if (px < 0) px = SEGUP - 1;                                  // idle items: the dummy slot
      sx[(0 * 2 + ih) * SEGUP + px] = hi;
      sx[(1 * 2 + ih) * SEGUP + px] = lo;
    };
    const int T2 = a.pairs * KS * KS / 2;                       // steps (pairs even)
    auto issue_w = [&](int st, int bw) __attribute__((always_inline)) {
      const f16x8* src = a.wpk + ((size_t)co_t * T2 + st) * WS2;
      f16x8* dst = smem + bw * WS2;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int q = (wave_u - LOADER_WAVES) * DPW + k;
        if (NP % DMA_WAVES == 0 || q < NP)
          __builtin_amdgcn_global_load_lds((const void*)(src + q * 64 + lane),
                                           (__attribute__((address_space(3))) void*)(dst + q * 64), 16, 0, 0);
      }
    };
    const int g = lane >> 4, r16 = lane & 15, gc = g & 1;
    const bool g_lo = g < 2;
    int rel16[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = min(m0 + wave_n * 64 + j * 16 + r16, mlast);
      const int y = m / a.W, x = m - y * a.W;
      rel16[j] = (y + a.in_pad) * Wi + x + a.in_pad - La;
    }
    f32x4 acc4[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc4[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments of the 4 pixel blocks held, A streamed per channel block
    auto mfma4x4 = [&](const f16x8* w, const f16x8 (&B)[4]) __attribute__((always_inline)) {
      f16x8 A = w[0];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f16x8 An = w[16 * (i < 3 ? i + 1 : 3)];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B[j], acc4[i][j], 0, 0, 0);
        A = An;
      }
    };
    const f16x8* wlane = smem + wave_m * 64 + r16;
    const f16x8* xlane = smem + 2 * WS2 + gc * SEGUP;
    // tap tau of the sequence -> its input offset (pair run, row, column) in units
    auto tap_off = [&](int tau) __attribute__((always_inline)) {
      const int p = tau / 9, r = tau - 9 * p, ky = r / 3, kx = r - 3 * ky;
      return (p & 1) * XSLABU + ky * Wi + kx;
    };
    // prologue: weights of step 0, the whole union run of pair 0
    if (!loader) issue_w(0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      load_q(0, q);
      store_q(q, 0);
    }
    __syncthreads();
    for (int st = 0; st < T2; ++st) {
      const int bw = st & 1;
      const int o0 = __builtin_amdgcn_readfirstlane(tap_off(2 * st));
      const int o1 = __builtin_amdgcn_readfirstlane(tap_off(2 * st + 1));
      const int cyc = st / 9, j9 = st - 9 * cyc;
      // staging of this step: a quarter of pair 2 cyc + 1 (steps 0-3) or 2 cyc + 2 (5-8)
      const int spair = j9 < 4 ? 2 * cyc + 1 : 2 * cyc + 2, sq = j9 < 4 ? j9 : j9 - 5;
      const bool stage = loader && j9 != 4 && spair < a.pairs;
      if (!loader && st + 1 < T2) issue_w(st + 1, bw ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      {   // M of the first tap
        f16x8 B[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) B[j] = xlane[o0 + rel16[j]];
        mfma4x4(wlane + bw * WS2 + g * BCO, B);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (stage) load_q(spair, sq);
      __builtin_amdgcn_sched_barrier(0);
      {   // M of the second tap
        f16x8 B[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) B[j] = xlane[o1 + rel16[j]];
        mfma4x4(wlane + bw * WS2 + (4 + g) * BCO, B);
      }
      __builtin_amdgcn_sched_barrier(0);
      {   // X of both taps: lanes g < 2 the first, g >= 2 the second
        const int ox = g_lo ? o0 : o1;
        f16x8 B[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) B[j] = xlane[2 * SEGUP + ox + rel16[j]];
        mfma4x4(wlane + bw * WS2 + ((g_lo ? 0 : 4) + gc) * BCO, B);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (stage) store_q(sq, spair & 1);
      __syncthreads();
    }
    // epilogue of the 16x16 blocks: lane = pixel r16 of block j, channels 4g..4g+3 of block i
    const int Wo = a.hpool ? a.W / 2 : a.W + 2 * a.out_pad;
    float* out_f = a.out + (size_t)n * a.out_fs;
    bool bad = false;
    float* ebias = (float*)smem;                  // [BCO] bias, [BCO] slope
    for (int i = tid; i < BCO; i += NT) {         // the K loop ended on a barrier: LDS is free
      ebias[i] = a.bias[co_t * BCO + i];
      ebias[BCO + i] = a.act == ACT_PRELU ? a.slope[co_t * BCO + i] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wave_n * 64 + j * 16 + r16;
      if (m > mlast) continue;
      const int y = m / a.W, x = m - y * a.W;
      float* op = a.hpool ? out_f + (size_t)(y * Wo + (x >> 1)) * 8
                          : out_f + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = wave_m * 64 + i * 16 + 4 * g, co = co_t * BCO + cl;
        const f32x4 b = *(const f32x4*)(ebias + cl);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc4[i][j][e] * a.wscale_inv + b[e];
        if (a.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (a.act == ACT_PRELU) {
          const f32x4 sl = *(const f32x4*)(ebias + BCO + cl);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) bad |= !(__builtin_fabsf(v[e]) < 65504.f);
        if (a.hpool) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = fmaxf(v[e], __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[e]), 0xB1, 0xF, 0xF, false)));
          if (x & 1) continue;
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
    if (bad) atomicOr(a.range_flag, 1);
    return;
  } else if constexpr (UNION) {
    // Row union, role split.  The KS input rows of a chunk pair are staged once, as
    // one run covering rows -P..+P of the tile, a third per ky step (ky then only
    // offsets the B reads by ky*Wi); for tiles spanning several image rows (46x82,
    // 92x164) that stages 2-2.5x fewer input bytes than one run per (pair, ky).
    // Issuing every wave's loads and DMA pieces at the top of a step stalled all 16
    // waves on the CU's vector-memory issue (~1.6k cycles per step, s_memtime
    // stamps) before any reached its MFMAs; here waves 0-9 (the threads < third)
    // stage the input union, waves 10-15 stream the weight slab, and both issue
    // between MFMA groups: the DMA of step t+1 ahead of the kx = 0 group, the input
    // loads of the next pair after it (+2-4 % per layer over issuing both at the top).
    static_assert(NWAVES == 16, "role split sized for 16-wave blocks");
    constexpr int LOADER_WAVES = 10, DMA_WAVES = NWAVES - LOADER_WAVES;
    constexpr int NP = WSLAB / 64;                               // 1 KiB DMA pieces per step
    constexpr int DPW = (NP + DMA_WAVES - 1) / DMA_WAVES;
    const bool loader = wave_u < LOADER_WAVES;
    const int Pw = P * Wi;
    const int segu = Lb - La + 2 * Pw + 2 * P + 1;        // rows -P..+P of the tile, one run
    const long long ubase = (long long)La - Pw - P;
    const int third = (2 * segu + KS - 1) / KS;           // staging items per ky step (<= 640)
    f32x4 ru[2];
    int c_ih[KS], c_px[KS];
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      const int it = ky * third + tid;
      const bool ok = tid < third && it < 2 * segu;
      c_ih[ky] = ok && it >= segu ? 1 : 0;
      c_px[ky] = ok ? it - c_ih[ky] * segu : -1;
    }
    auto load_c = [&](int c2, int ky) __attribute__((always_inline)) {
      if (c_px[ky] >= 0) {
        const int c = min(2 * c2 + c_ih[ky], a.cin_chunks - 1);
        if constexpr (VIN) {   // padded (row, column) of the item, recomputed (no registers held across the loop)
          const int u = (int)ubase + c_px[ky], yy = x3_div(u, inv_wi);
          float4 l4, h4;
          x3_vin_load(in_f + (size_t)c * a.in_chs, yy, u - yy * Wi, a, l4, h4);
          ru[0] = f32x4{l4.x, l4.y, l4.z, l4.w};
          ru[1] = f32x4{h4.x, h4.y, h4.z, h4.w};
        } else {
          const float* src = in_f + (size_t)c * a.in_chs + (size_t)(ubase + c_px[ky]) * 8;
          ru[0] = *(const f32x4*)src;
          ru[1] = *(const f32x4*)(src + 4);
        }
      }
    };
    auto store_c = [&](int c2, int ky, int bx) __attribute__((always_inline)) {
      f16x8* sx = smem + 2 * WSLAB + bx * XSLABU;
      // a missing odd chunk stages the last real chunk again (load_c clamps): its packed
      // weights are zero (pack_x3), and the staged values are finite (range-checked), so
      // it adds exact zeros
      f16x8 hi, lo;
      x3_split8(ru[0], ru[1], hi, lo);
      const int px = c_px[ky] < 0 ? SEGUP - 1 : c_px[ky];   // idle items: the dummy slot
      sx[(0 * 2 + c_ih[ky]) * SEGUP + px] = hi;
      sx[(1 * 2 + c_ih[ky]) * SEGUP + px] = lo;
    };
    auto issue_c = [&](int t, int bw) __attribute__((always_inline)) {
      const f16x8* src = a.wpk + ((size_t)co_t * T + t) * WSLAB;
      f16x8* dst = smem + bw * WSLAB;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int q = (wave_u - LOADER_WAVES) * DPW + k;
        if (NP % DMA_WAVES == 0 || q < NP)
          __builtin_amdgcn_global_load_lds((const void*)(src + q * 64 + lane),
                                           (__attribute__((address_space(3))) void*)(dst + q * 64), 16, 0, 0);
      }
    };
    auto tap_u = [&](int bw, int bx, int ky, int kx) __attribute__((always_inline)) {
      tap(smem + bw * WSLAB + h * BCO + wave_m * WM * 32 + l32,
          smem + 2 * WSLAB + bx * XSLABU + h * SEGUP + ky * Wi, SEGUP, kx);
    };
    // prologue: weights of step 0, the whole union of pair 0
    if (!loader) issue_c(0, 0);
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      load_c(0, ky);
      store_c(0, ky, 0);
    }
    __syncthreads();
    for (int c2 = 0; c2 < a.pairs; ++c2) {
      const bool next = c2 + 1 < a.pairs;
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const int t = c2 * KS + ky;
        auto stamp = [&](int k) __attribute__((always_inline)) {
          if constexpr (STAMP) {
            if (blockIdx.x == 0 && lane == 0) a.dbg[((size_t)wave * T + t) * 4 + k] = __builtin_amdgcn_s_memtime();
          }
        };
        stamp(0);
        if constexpr (STAMP) {
          // clock check: s_memrealtime (100 MHz) beside s_memtime at steps 1 and T-1, slots past the stamps
          if (blockIdx.x == 0 && lane == 0 && wave == 0 && (t == 1 || t == T - 1)) {
            a.dbg[(size_t)16 * T * 4 + (t == 1 ? 0 : 2)] = __builtin_amdgcn_s_memtime();
            a.dbg[(size_t)16 * T * 4 + (t == 1 ? 1 : 3)] = __builtin_amdgcn_s_memrealtime();
          }
        }
        if (!loader && t + 1 < T) issue_c(t + 1, (t + 1) & 1);
        stamp(1);
        __builtin_amdgcn_sched_barrier(0);
        tap_u(t & 1, c2 & 1, ky, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (loader && next) load_c(c2 + 1, ky);   // a third of the next pair's union per step
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kx = 1; kx < KS; ++kx) tap_u(t & 1, c2 & 1, ky, kx);
        __builtin_amdgcn_sched_barrier(0);
        stamp(2);
        if (loader && next) store_c(c2 + 1, ky, (c2 + 1) & 1);
        stamp(3);
        __syncthreads();
      }
    }
  } else {
    // Generic loop: one step = (pair, ky); weights by LDS-DMA one step ahead, the
    // input row run register-staged one step ahead.
    int ih[IT], ipx[IT];                 // staging items: tid_g + i*NTG -> (chunk of the step, pixel)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int it = tid_g + i * NTG;
      ih[i] = min(it / seg, 2 * PPS - 1);
      ipx[i] = it - ih[i] * seg;
      if (it >= 2 * PPS * seg) ipx[i] = -1;   // idle
    }
    f32x4 raw[IT][2];
    bool fold_bad = false;
    auto load_x = [&](int t) __attribute__((always_inline)) {
      const int c2 = t / KS, ky = t - c2 * KS;
      const long long row = (long long)(La + (ky - P) * Wi - P);
      X3Fold fe[2];
      if constexpr (FOLD) {   // the step's two chunks (uniform)
        fe[0] = a.fold[min(2 * c2, a.cin_chunks - 1)];
        fe[1] = a.fold[min(2 * c2 + 1, a.cin_chunks - 1)];
      }
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        const int c = 2 * PPS * c2 + ih[i];
        if (ipx[i] >= 0 && c < a.cin_chunks) {
          if (FOLD && (ih[i] ? fe[1].ws : fe[0].ws)) {
            // x3_splitk_reduce's arithmetic on the producer's partials: ranges summed in
            // order, x 2^-s + bias, activation (the same bits it would have stored); the
            // padding ring reads as zeros; the value is range-checked here
            const X3Fold& f = ih[i] ? fe[1] : fe[0];
            const int u = (int)row + ipx[i], yy = x3_div(u, inv_wi), y = yy - a.in_pad, x = u - yy * Wi - a.in_pad;
            if (y < 0 || y >= a.H || x < 0 || x >= a.W) {
              raw[i][0] = raw[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
              const float* p = f.ws + (size_t)n * f.fstride + (size_t)(y * a.W + x) * 8;
              // every range's partial in flight at once (S <= 8, uniform), then the sum in
              // range order
              f32x4 q0[8], q1[8];
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const float* pk = p + (k < f.S ? k : 0) * f.sstride;
                q0[k] = *(const f32x4*)pk;
                q1[k] = *(const f32x4*)(pk + 4);
              }
              // x3_canonical_order: the two halves of the ranges, each in order, then added
              const int hh = (f.S + 1) / 2;
              f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, u0 = s0, u1 = s0;
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                if (k < hh) {
                  s0 += q0[k];
                  s1 += q1[k];
                } else if (k < f.S) {
                  u0 += q0[k];
                  u1 += q1[k];
                }
              }
              if (f.S > hh) {
                s0 += u0;
                s1 += u1;
              }
              const f32x4 b0 = *(const f32x4*)f.bias, b1 = *(const f32x4*)(f.bias + 4);
              f32x4 v0, v1;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v0[e] = s0[e] * f.scale + b0[e];
                v1[e] = s1[e] * f.scale + b1[e];
              }
              if (f.act == ACT_RELU) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  v0[e] = v0[e] > 0.f ? v0[e] : 0.f;
                  v1[e] = v1[e] > 0.f ? v1[e] : 0.f;
                }
              } else if (f.act == ACT_PRELU) {
                const f32x4 l0 = *(const f32x4*)f.slope, l1 = *(const f32x4*)(f.slope + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  v0[e] = v0[e] >= 0.f ? v0[e] : v0[e] * l0[e];
                  v1[e] = v1[e] >= 0.f ? v1[e] : v1[e] * l1[e];
                }
              }
#pragma unroll
              for (int e = 0; e < 4; ++e) fold_bad |= !(__builtin_fabsf(v0[e]) < 65504.f) || !(__builtin_fabsf(v1[e]) < 65504.f);
              raw[i][0] = v0;
              raw[i][1] = v1;
            }
          } else if constexpr (VIN) {   // padded (row, column) of the item, recomputed per step
            const int u = (int)row + ipx[i], yy = x3_div(u, inv_wi);
            float4 l4, h4;
            x3_vin_load(in_f + (size_t)c * a.in_chs, yy, u - yy * Wi, a, l4, h4);
            raw[i][0] = f32x4{l4.x, l4.y, l4.z, l4.w};
            raw[i][1] = f32x4{h4.x, h4.y, h4.z, h4.w};
          } else {
            const float* src = in_f + (size_t)c * a.in_chs + (size_t)(row + ipx[i]) * 8;
            raw[i][0] = *(const f32x4*)src;
            raw[i][1] = *(const f32x4*)(src + 4);
          }
        } else {
          raw[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
          raw[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    };
    // VAR 32: each K group on its own pair of buffers
    f16x8* const gsm = smem + grp * 2 * BUF;
    auto wbuf = [&](int buf) __attribute__((always_inline)) { return gsm + buf * (SIB || DEEP ? WSLAB : BUF); };
    auto xbuf = [&](int buf) __attribute__((always_inline)) {
      return SIB ? gsm + 2 * WSLAB : DEEP ? gsm + 3 * WSLAB + buf * XSLAB : gsm + buf * BUF + WSLAB;
    };
    auto store_x = [&](int buf) __attribute__((always_inline)) {
      f16x8* s = xbuf(buf);
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        if (ipx[i] < 0) continue;
        f16x8 hi, lo;
        x3_split8(raw[i][0], raw[i][1], hi, lo);
        s[(0 * 2 * PPS + ih[i]) * SEGP + ipx[i]] = hi;
        s[(1 * 2 * PPS + ih[i]) * SEGP + ipx[i]] = lo;
      }
    };
    auto issue_w = [&](int t, int buf) __attribute__((always_inline)) {
      // HALFCO: the 128-channel packing, rows of 128 units; this block takes half of each
      const f16x8* src = HALFCO ? a.wpk + ((size_t)(co_t >> 1) * T + t) * (2 * WSLAB) + (co_t & 1) * 64
                                : a.wpk + ((size_t)co_t * T + t) * WSLAB;
      f16x8* dst = wbuf(buf);
#pragma unroll
      for (int q0 = 0; q0 < WSLAB / 64; q0 += NWAVES) {
        const int q = q0 + wave_u;
        if ((WSLAB / 64) % NWAVES == 0 || q < WSLAB / 64) {
          const f16x8* sp = src + q * (HALFCO ? 128 : 64);
          if constexpr (PPS == 2 && KS > 1) {
            // step (pair pair c2, ky): row ky of pairs 2 c2 and 2 c2 + 1, not adjacent in the
            // [pair][ky][kx] packing -- piece q of the slab from pair 2 c2 + q / NP1
            constexpr int NP1 = WSLAB1 / 64;
            const int c2 = t / KS, ky = t - c2 * KS, pp = q / NP1;
            sp = a.wpk + (((size_t)co_t * a.pairs + 2 * c2 + pp) * KS + ky) * WSLAB1 + (q - pp * NP1) * 64;
          }
          __builtin_amdgcn_global_load_lds((const void*)(sp + lane),
                                           (__attribute__((address_space(3))) void*)(dst + q * 64), 16, 0, 0);
        }
      }
    };
    auto compute = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int pp = 0; pp < PPS; ++pp) {
        const f16x8* sw = wbuf(buf) + pp * WSLAB1 + h * BCO + wave_m * WM * 32 + l32;
        const f16x8* sx = xbuf(buf) + (2 * pp + h) * SEGP;
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) tap(sw, sx, PPS * SEGP, kx);
      }
    };
    auto compute_deep = [&](int wb, int xb) __attribute__((always_inline)) {
      const f16x8* sw = wbuf(wb) + h * BCO + wave_m * WM * 32 + l32;
      const f16x8* sx = xbuf(xb) + h * SEGP;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) tap(sw, sx, SEGP, kx);
    };
    // K ranges: [t0, t1) of this block (SPLIT: one range; G2: this group's half), range
    // length R steps, the first range of the second half at step th
    int t0 = 0, t1 = T, R = T, th = T;
    if constexpr (SPLIT || RANGED) {
      // PPS == 2: the host checks that every range has an even number of pairs
      const int pps = (a.pairs + a.ksplit - 1) / a.ksplit;
      R = pps / PPS * KS;
      th = min(T, (a.ksplit + 1) / 2 * R);
      if constexpr (SPLIT) {
        t0 = ks_i * R;
        t1 = min(a.pairs, (ks_i + 1) * pps) / PPS * KS;
      }
      if constexpr (G2) {
        t0 = grp ? th : 0;
        t1 = grp ? T : th;
      }
    }
    // x3_canonical_order: each half's range sums (each from zero) added in order onto +0, then
    // the halves added; tot holds the first half (G2: this group's half), toth the second
    f32x16 tot[RANGED ? WM : 1][RANGED ? WN : 1];
    f32x16 toth[RANGED && !G2 ? WM : 1][RANGED && !G2 ? WN : 1];
    if constexpr (RANGED) {
#pragma unroll
      for (int wm = 0; wm < WM; ++wm)
#pragma unroll
        for (int wn = 0; wn < WN; ++wn)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            tot[wm][wn][r] = 0.f;
            if constexpr (!G2) toth[wm][wn][r] = 0.f;
          }
    }
    auto range_end = [&](int t) __attribute__((always_inline)) {
      if constexpr (RANGED) {
        if (t + 1 == t1 || (t + 1) % R == 0) {
          if (!G2 && t >= th) {                        // (uniform) a range of the second half
            if constexpr (!G2) {
#pragma unroll
              for (int wm = 0; wm < WM; ++wm)
#pragma unroll
                for (int wn = 0; wn < WN; ++wn) toth[wm][wn] += acc[wm][wn];
            }
          } else {
#pragma unroll
            for (int wm = 0; wm < WM; ++wm)
#pragma unroll
              for (int wn = 0; wn < WN; ++wn) tot[wm][wn] += acc[wm][wn];
          }
#pragma unroll
          for (int wm = 0; wm < WM; ++wm)
#pragma unroll
            for (int wn = 0; wn < WN; ++wn)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[wm][wn][r] = 0.f;
        }
      }
    };
    if constexpr (DEEP) {
      // Role split (as the row union's): loader waves [0, NL) register-stage the input runs
      // two steps ahead and write the split run of step t + 1 at the end of step t; DMA
      // waves [NL, NWAVES) stream the weight slabs two steps ahead into a ring of three.
      // No wave does both, so hipcc never drains a loader's loads in front of its LDS
      // writes (the LDS-DMA aliasing rule); the DMA waves wait with a counted vmcnt, and the
      // block meets at a raw s_barrier (__syncthreads would drain every DMA in flight).
      constexpr int NL = NWAVES / 2, ND = NWAVES - NL;
      constexpr int NP = WSLAB / 64, DPW = (NP + ND - 1) / ND;     // weight pieces, per DMA wave
      constexpr int ITL = (2 * SEGMAX + NL * 64 - 1) / (NL * 64);   // staging items per loader thread
      const bool loader = wave_u < NL;
      int lih[ITL], lpx[ITL];
#pragma unroll
      for (int k = 0; k < ITL; ++k) {
        const int it = tid + k * NL * 64;
        lih[k] = min(it / seg, 1);
        lpx[k] = loader && it < 2 * seg ? it - lih[k] * seg : -1;
      }
      f32x4 rs[2][ITL][2];                                          // two register slots
      // Every load and store is unconditional (idle items read pixel 0 and write the dummy
      // slot; past the last step the loads and DMAs repeat the last step's), so the number of
      // vector-memory operations in flight is the same on every path and hipcc's wait-count
      // pass keeps the younger slot's loads in flight (counted vmcnt) instead of draining them.
      auto dload = [&](int t, int sl) __attribute__((always_inline)) {
        t = min(t, t1 - 1);
        const int c2 = t / KS, ky = t - c2 * KS;
        const long long row = (long long)(La + (ky - P) * Wi - P);
#pragma unroll
        for (int k = 0; k < ITL; ++k) {
          // a missing odd chunk stages the last real one (its packed weights are zero)
          const int c = min(2 * c2 + lih[k], a.cin_chunks - 1);
          const float* src = in_f + (size_t)c * a.in_chs + (size_t)(row + max(lpx[k], 0)) * 8;
          rs[sl][k][0] = *(const f32x4*)src;
          rs[sl][k][1] = *(const f32x4*)(src + 4);
        }
      };
      auto dstore = [&](int xb, int sl) __attribute__((always_inline)) {
        f16x8* sx = xbuf(xb);
#pragma unroll
        for (int k = 0; k < ITL; ++k) {
          f16x8 hi, lo;
          x3_split8(rs[sl][k][0], rs[sl][k][1], hi, lo);
          const int px = lpx[k] < 0 ? SEGP - 1 : lpx[k];
          sx[(0 * 2 + lih[k]) * SEGP + px] = hi;
          sx[(1 * 2 + lih[k]) * SEGP + px] = lo;
        }
      };
      auto dissue = [&](int t, int wb) __attribute__((always_inline)) {
        t = min(t, t1 - 1);
        const f16x8* src = HALFCO ? a.wpk + ((size_t)(co_t >> 1) * T + t) * (2 * WSLAB) + (co_t & 1) * 64
                                  : a.wpk + ((size_t)co_t * T + t) * WSLAB;
        f16x8* dst = wbuf(wb);
#pragma unroll
        for (int k = 0; k < DPW; ++k) {
          // every DMA wave issues DPW pieces (a spare repeats the last piece: the same bytes
          // to the same place), so the counted wait below is exact
          const int q = min((wave_u - NL) * DPW + k, NP - 1);
          __builtin_amdgcn_global_load_lds((const void*)(src + q * (HALFCO ? 128 : 64) + lane),
                                           (__attribute__((address_space(3))) void*)(dst + q * 64), 16, 0, 0);
        }
      };
      // the whole loop once per role (ROLE: the loader's), so hipcc's wait-count pass never
      // merges a DMA in flight into a loader's path (it would drain before its LDS writes)
      auto run = [&](auto role) __attribute__((always_inline)) {
        constexpr bool LOADER = decltype(role)::value;
        // this wave's DMA of the next step has landed (`later`: one more step of pieces may
        // stay in flight), its LDS writes are done, then the block barrier
        auto wait_barrier = [&](bool later) __attribute__((always_inline)) {
          if constexpr (!LOADER) {
            if (later) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        };
        if constexpr (LOADER) {
          dload(t0, 0);
          dload(t0 + 1, 1);
          dstore(0, 0);
        } else {
          dissue(t0, 0);
          dissue(t0 + 1, 1);
        }
        wait_barrier(true);
        // step t (i = t - t0): weights in ring buffer i % 3, input in buffer i & 1 from
        // register slot i & 1; it stages step t + 2 into what step t - 1 used
        auto step = [&](int t, int sl) __attribute__((always_inline)) {
          const int i = t - t0;
          if constexpr (LOADER) dload(t + 2, sl);
          else dissue(t + 2, (i + 2) % 3);
          __builtin_amdgcn_sched_barrier(0);
          compute_deep(i % 3, sl);
          range_end(t);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (LOADER) dstore(sl ^ 1, sl ^ 1);
          wait_barrier(true);
        };
        for (int t = t0; t < t1; t += 2) {
          step(t, 0);
          if (t + 1 < t1) step(t + 1, 1);
        }
        // the spare DMAs past the last step land before the epilogue reuses the LDS
        wait_barrier(false);
      };
      if (loader) run(std::true_type{});
      else run(std::false_type{});
    } else {
#ifdef ISLPOSE_DEV
    // timing-only ablations (tools/convbench, ISLPOSE_X3_ABL bits): 1 no compute, 2 no input
    // staging, 4 no weight DMA, 8 no barrier, 16 no prologue staging (the epilogue bits 32 / 64
    // are read there) -- wrong results, development build only
    const int abl = a.abl;
#else
    constexpr int abl = 0;
#endif
    if (!(abl & 16)) {
      issue_w(t0, 0);
      load_x(t0);
      store_x(0);
    }
    __syncthreads();
    // G2: both groups meet at every barrier; the first group has at least as many steps (its
    // half holds the larger share of the ranges), the second idles through the surplus
    const int nsteps = G2 ? th : t1 - t0;
    for (int i = 0; i < nsteps; ++i) {
      const int t = t0 + i;
      const bool on = !G2 || t < t1;                // (uniform per group)
      const int buf = i & 1;
      if (on && t + 1 < t1) {
        if (!(abl & 4)) issue_w(t + 1, buf ^ 1);
        if (!(abl & 2)) load_x(t + 1);
      }
      if (on) {
        if (!(abl & 1)) compute(buf);
        range_end(t);
      }
      if constexpr (SIB) __syncthreads();         // every wave is done with the one input buffer
      if (on && t + 1 < t1 && !(abl & 2)) store_x(buf ^ 1);
      if (!(abl & 8)) __syncthreads();
    }
    }
    if constexpr (G2) {
      // the second group's half through LDS (the loop ended on a barrier), added to the first
      // group's in the first group's waves: lo + hi
      float* xch = (float*)smem;
      constexpr int NV = WM * WN * 16;
      if (grp) {
#pragma unroll
        for (int wm = 0; wm < WM; ++wm)
#pragma unroll
          for (int wn = 0; wn < WN; ++wn)
#pragma unroll
            for (int r = 0; r < 16; ++r) xch[((size_t)wave_g * NV + (wm * WN + wn) * 16 + r) * 64 + lane] = tot[wm][wn][r];
      }
      __syncthreads();
      if (!grp) {
#pragma unroll
        for (int wm = 0; wm < WM; ++wm)
#pragma unroll
          for (int wn = 0; wn < WN; ++wn)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              acc[wm][wn][r] = tot[wm][wn][r] + xch[((size_t)wave_g * NV + (wm * WN + wn) * 16 + r) * 64 + lane];
      }
      __syncthreads();                              // the epilogue reuses the LDS
    } else if constexpr (RANGED) {
      const bool two = a.ksplit > (a.ksplit + 1) / 2;   // a second half exists (S >= 2)
#pragma unroll
      for (int wm = 0; wm < WM; ++wm)
#pragma unroll
        for (int wn = 0; wn < WN; ++wn) acc[wm][wn] = two ? tot[wm][wn] + toth[wm][wn] : tot[wm][wn];
    }
    if constexpr (FOLD) {
      if (fold_bad) atomicOr(a.range_flag, 1);
    }
  }

  if constexpr (SPLIT) {
    // this range's sum (unscaled, as the in-block ranges keep it) into its slice of
    // the workspace; the workspace carries round8(cout) channels, so the 4-channel
    // groups never overrun
    const size_t plane = (size_t)HW * 8;
    float* wsb = a.ws + ((size_t)ks_i * a.nfr + n) * (size_t)((a.cout + 7) / 8) * plane;
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) {
      const int m = m0 + (wave_n * WN + wn) * 32 + l32;
      if (m > mlast) continue;
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) {
        const int cob = co_t * BCO + (wave_m * WM + wm) * 32 + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co = cob + 8 * q;
          if (co >= a.cout) continue;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[wm][wn][4 * q + e];
          *(f32x4*)(wsb + (size_t)(co >> 3) * plane + (size_t)m * 8 + (co & 7)) = v;
        }
      }
    }
    return;
  }
  if constexpr (FUSE67) {
    // Mconv6 -> Mconv7 (model.py:108-109, 125-126: two 1x1 convs, Mconv6 + PReLU, Mconv7).
    // This block holds all BCO Mconv6 channels of its BPX pixels: wave (wave_m, wave_n) the
    // channels [64 wave_m, 64 wave_m + 64) of pixel tiles wave_n * WN + wn.  One pass per wn
    // (the pixel tiles wave_n * WN + wn of every wave_n): Mconv6's epilogue and split, each
    // wave's Mconv7 sums into LDS, then the waves' sums added in wave order and stored.
    static_assert(KS == 1 && WM == 2 && WN == 2 && !SPLIT && !RANGED && !UNION && !DEEP && !VIN && !HALFCO,
                  "fused 1x1 pair: generic loop, 64co x 64px waves");
#ifdef ISLPOSE_DEV
    // ablations (tools/archive/cb_f67.sh): 64 no epilogue, 32 Mconv7 filters not loaded
    if (a.abl & 64) return;
    const bool abl_f7 = (a.abl & 32) != 0;
#else
    constexpr bool abl_f7 = false;
#endif
    constexpr int RPX = WAVES_N * 32;            // pixels of one pass
    float* eb = (float*)smem;                    // [BCO] bias6, [BCO] slope6, [64] bias7, [64] slope7
    float* red = eb + 2 * BCO + 128;             // [WAVES_M][RPX][F7_ROWS]
    for (int i = tid; i < BCO; i += NT) {        // the K loop ended on a barrier: LDS is free
      eb[i] = a.bias[i];
      eb[BCO + i] = a.act == ACT_PRELU ? a.slope[i] : 0.f;
    }
    for (int i = tid; i < 64; i += NT) {
      eb[2 * BCO + i] = i < a.cout7 ? a.bias7[i] : 0.f;
      eb[2 * BCO + 64 + i] = i < a.cout7 && a.act7 == ACT_PRELU ? a.slope7[i] : 0.f;
    }
    __syncthreads();
    bool bad = false;
    const int nt7 = (a.cout7 + 31) / 32;         // Mconv7 row tiles (1 or 2)
    const int nch = (a.cout7 + 7) / 8;           // its 8-channel output chunks
    constexpr int KB = BCO / 16;                 // Mconv7 K blocks (16 Mconv6 channels each)
    const float* bias7 = eb + 2 * BCO;
    const float* slope7 = eb + 2 * BCO + 64;
    const int Wo = a.W + 2 * a.out_pad;
    float* out_f = a.out + (size_t)n * a.out_fs;
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) {
      // Mconv6's epilogue (x 2^-s, bias, activation, range check) and the split: register r
      // of a 32x32 D tile is row (r & 3) + 8 (r >> 2) + 4 h, so registers 8 kq .. 8 kq + 7 of
      // lane half h are the K = 16 B fragment of rows {16 kq + 4 h + 8 (j >> 2) + (j & 3)};
      // Mconv7's filters are packed in that K order (pack_x3_f7): no value leaves its lane
      const bool live = m0 + (wave_n * WN + wn) * 32 + l32 <= mlast;
      f16x8 Bh[WM][2], Bl[WM][2];
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) {
        f32x16 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = (wave_m * WM + wm) * 32 + 4 * h + 8 * q;
          const f32x4 b = *(const f32x4*)(eb + col);
          const f32x4 sl = *(const f32x4*)(eb + BCO + col);
          // (the activation chosen once per 4 registers: a test per register made a scalar branch
          // chain of the whole split)
          f32x4 x;
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = acc[wm][wn][4 * q + e] * a.wscale_inv + b[e];
          if (a.act == ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = x[e] > 0.f ? x[e] : 0.f;
          } else if (a.act == ACT_PRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = x[e] >= 0.f ? x[e] : x[e] * sl[e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bad |= live && !(__builtin_fabsf(x[e]) < 65504.f);
            v[4 * q + e] = x[e];
          }
        }
#pragma unroll
        for (int kq = 0; kq < 2; ++kq)
          x3_split8(f32x4{v[8 * kq], v[8 * kq + 1], v[8 * kq + 2], v[8 * kq + 3]},
                    f32x4{v[8 * kq + 4], v[8 * kq + 5], v[8 * kq + 6], v[8 * kq + 7]}, Bh[wm][kq], Bl[wm][kq]);
      }
      // this wave's 64-channel share of every Mconv7 row tile: its K blocks in order, 3 split
      // products each, from zero
      for (int t = 0; t < nt7; ++t) {
        f32x16 d;
#pragma unroll
        for (int r = 0; r < 16; ++r) d[r] = 0.f;
#pragma unroll
        for (int wm = 0; wm < WM; ++wm)
#pragma unroll
          for (int kq = 0; kq < 2; ++kq) {
            const int kb = (wave_m * WM + wm) * 2 + kq;
            const f16x8* wp = a.wpk7 + ((size_t)(t * KB + kb) * 2) * 64 + lane;
            const f16x8 Ah = abl_f7 ? Bh[wm][kq] : wp[0], Al = abl_f7 ? Bl[wm][kq] : wp[64];
            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bh[wm][kq], d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bl[wm][kq], d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(Al, Bh[wm][kq], d, 0, 0, 0);
          }
        float* rp = red + ((size_t)wave_m * RPX + wave_n * 32 + l32) * F7_ROWS + 32 * t + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) *(f32x4*)(rp + 8 * q) = f32x4{d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]};
      }
      __syncthreads();
      // the waves' sums added in wave order, x 2^-s, bias, activation, range check; one thread
      // per (8-channel output chunk, pixel): 32-byte stores, neighbouring pixels together
      for (int task = tid; task < nch * RPX; task += NT) {
        const int c8 = task / RPX, px = task - c8 * RPX;
        const int m = m0 + ((px >> 5) * WN + wn) * 32 + (px & 31);
        if (m > mlast) continue;
        // x3_canonical_order over the waves' shares (the K ranges of the two-launch Mconv7,
        // pack_x3_f7): each half from +0 in wave order, then the halves
        const float* rq = red + (size_t)px * F7_ROWS + 8 * c8;
        constexpr int HW7 = (WAVES_M + 1) / 2;
        f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0, u0 = s0, u1 = s0;
#pragma unroll
        for (int w = 0; w < WAVES_M; ++w) {
          const f32x4 p0 = *(const f32x4*)(rq + (size_t)w * RPX * F7_ROWS);
          const f32x4 p1 = *(const f32x4*)(rq + (size_t)w * RPX * F7_ROWS + 4);
          if (w < HW7) { s0 += p0; s1 += p1; }
          else { u0 += p0; u1 += p1; }
        }
        if constexpr (WAVES_M > HW7) { s0 += u0; s1 += u1; }
        const int co = 8 * c8;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (e < 4 ? s0[e] : s1[e - 4]) * a.wscale7_inv + bias7[co + e];
        if (a.act7 == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = o[e] > 0.f ? o[e] : 0.f;
        } else if (a.act7 == ACT_PRELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = o[e] >= 0.f ? o[e] : o[e] * slope7[co + e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) bad |= co + e < a.cout7 && !(__builtin_fabsf(o[e]) < 65504.f);
        const int y = m / a.W, x = m - y * a.W;
        float* oc = out_f + (size_t)(co >> 3) * a.out_chs + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8;
        if (co + 7 < a.cout7) {
          *(f32x4*)oc = f32x4{o[0], o[1], o[2], o[3]};
          *(f32x4*)(oc + 4) = f32x4{o[4], o[5], o[6], o[7]};
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (co + e < a.cout7) oc[e] = o[e];
        }
      }
      __syncthreads();                           // red is rewritten by the next pass
    }
    if (bad) atomicOr(a.range_flag, 1);
    return;
  }
  // epilogue: x 2^-s, bias + activation, range check, masked float4 stores.  Bias and
  // PReLU slopes come from LDS (staged once), so no global load -- and no vmcnt(0)
  // behind the stores issued so far -- sits between the output stores.
  const int Wo = a.hpool ? a.W / 2 : a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
  bool bad = false;
#ifdef ISLPOSE_DEV
  // ablations (tools/convbench, ISLPOSE_X3_ABL): 64 no epilogue at all, 32 no bias load
  if (a.abl & 64) return;
  const bool abl_bias = (a.abl & 32) != 0;
#else
  constexpr bool abl_bias = false;
#endif
  float* ebias = (float*)smem;                  // [BCO] bias, [BCO] slope
  for (int i = tid; i < BCO; i += NT) {         // the K loop ended on a barrier: LDS is free
    ebias[i] = abl_bias ? 0.f : a.bias[co_t * BCO + i];
    ebias[BCO + i] = !abl_bias && a.act == ACT_PRELU ? a.slope[co_t * BCO + i] : 0.f;
  }
  __syncthreads();
  if (G2 && grp) return;                        // the first K group stores the sums
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int m = m0 + (wave_n * WN + wn) * 32 + l32;
    if (m > mlast) continue;
    const int y = m / a.W, x = m - y * a.W;
    float* op = a.hpool ? out_f + (size_t)(y * Wo + (x >> 1)) * 8
                        : out_f + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8;
#pragma unroll
    for (int wm = 0; wm < WM; ++wm) {
      const int cob = co_t * BCO + (wave_m * WM + wm) * 32 + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = cob + 8 * q;
        const f32x4 b = *(const f32x4*)(ebias + co - co_t * BCO);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[wm][wn][4 * q + e] * a.wscale_inv + b[e];
        if (a.act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (a.act == ACT_PRELU) {
          const f32x4 sl = *(const f32x4*)(ebias + BCO + co - co_t * BCO);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) bad |= !(__builtin_fabsf(v[e]) < 65504.f);
        if (a.hpool) {
          // pixels m, m+1 (x even, x+1: W even, tiles start on even pixels) sit in lanes
          // l, l^1: take the pair's max, the even lane stores it
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = fmaxf(v[e], __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[e]), 0xB1, 0xF, 0xF, false)));
          if (x & 1) continue;
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
  if (bad) atomicOr(a.range_flag, 1);
}

// ---------------------------------------------------------------------------
// conv1_1 of every net: 3 input channels, 3x3, 64 outputs.  Through the generic
// kernel a pixel costs 9 pair-taps of K = 16 for 27 real products (5.3x the work);
// here K is the 27 real (ky, kx, c) values padded to 32 -- two MFMA K-steps --
// from an im2col tile of 256 pixels x 32 k in LDS (fp16 hi | lo, 32 KiB), built
// straight from the padded input.  Weights [kk][hi|lo][h][64][8], k = 16 kk + 8 h
// + j = 9 ky + 3 kx + c (host: pack_x3_rgb), scaled by 2^s as pack_x3.  The layer
// is then bound by its 64-channel fp32 output write (~4.1 TB/s of HBM traffic).  4 waves,
// 64co x 64px each.
// ---------------------------------------------------------------------------
constexpr int RGB_BCO = 64, RGB_TILE = 256;

// the variant of the last conv_x3 / conv_x3_rgb launch of this thread (x3_last_variant)
static thread_local int t_last_variant = 0;
int x3_last_variant() { return t_last_variant; }

template <int RGB_BPX>
__global__ void __launch_bounds__(RGB_BPX, 1) conv_x3_rgb(X3Args a) {
  constexpr int RGB_NT = RGB_BPX;
  __shared__ f16x8 s_x[2][4][RGB_BPX];          // [hi|lo][k chunk q][px]
  __shared__ f16x8 s_w[2][2][2][RGB_BCO];        // [kk][hi|lo][h][co]
  __shared__ float s_b[2 * RGB_BCO];             // bias, PReLU slope
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  int bid = blockIdx.x;
  {
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int pt = bid % a.px_tiles, n = bid / a.px_tiles;
  const int HW = a.H * a.W, m0 = pt * RGB_BPX, mlast = min(m0 + RGB_BPX, HW) - 1;
  const int Wi = a.W + 2 * a.in_pad;
  const float* in_f = a.in + (size_t)n * a.in_fs;
  for (int i = tid; i < 2 * 2 * 2 * RGB_BCO; i += RGB_NT) (&s_w[0][0][0][0])[i] = a.wpk[i];
  for (int i = tid; i < RGB_BCO; i += RGB_NT) {
    s_b[i] = a.bias[i];
    s_b[RGB_BCO + i] = a.act == ACT_PRELU ? a.slope[i] : 0.f;
  }
  _Float16* sxh = (_Float16*)&s_x[0][0][0];
  auto put = [&](int hl, int k, int px, _Float16 v) __attribute__((always_inline)) {
    sxh[(((size_t)hl * 4 + (k >> 3)) * RGB_BPX + px) * 8 + (k & 7)] = v;
  };
  // im2col: task (px, ky) reads the 3 input pixels kx = 0..2 of kernel row ky
  for (int task = tid; task < 3 * RGB_BPX; task += RGB_NT) {
    const int ky = task / RGB_BPX, px = task - ky * RGB_BPX;
    const int m = min(m0 + px, mlast);
    const int y = m / a.W, x = m - y * a.W;
    const float* src = in_f + (size_t)((y + ky - 1 + a.in_pad) * Wi + x - 1 + a.in_pad) * 8;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const f32x4 v = *(const f32x4*)(src + kx * 8);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = 9 * ky + 3 * kx + c;
        const _Float16 hi = (_Float16)v[c];
        put(0, k, px, hi);
        put(1, k, px, (_Float16)(v[c] - (float)hi));
      }
    }
  }
  for (int px = tid; px < RGB_BPX; px += RGB_NT)
#pragma unroll
    for (int k = 27; k < 32; ++k) {
      put(0, k, px, (_Float16)0.f);
      put(1, k, px, (_Float16)0.f);
    }
  __syncthreads();
  f32x16 acc[2][2];
#pragma unroll
  for (int wm = 0; wm < 2; ++wm)
#pragma unroll
    for (int wn = 0; wn < 2; ++wn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[wm][wn][r] = 0.f;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    f16x8 A[2][2], B[2][2];
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
#pragma unroll
      for (int wm = 0; wm < 2; ++wm) A[wm][hl] = s_w[kk][hl][h][wm * 32 + l32];
#pragma unroll
      for (int wn = 0; wn < 2; ++wn) B[wn][hl] = s_x[hl][2 * kk + h][wave * 64 + wn * 32 + l32];
    }
#pragma unroll
    for (int wm = 0; wm < 2; ++wm)
#pragma unroll
      for (int wn = 0; wn < 2; ++wn) {
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[wn][0], acc[wm][wn], 0, 0, 0);
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][0], B[wn][1], acc[wm][wn], 0, 0, 0);
        acc[wm][wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[wm][1], B[wn][0], acc[wm][wn], 0, 0, 0);
      }
  }
  // epilogue (as conv_x3_f16's): x 2^-s, bias, activation, range check, float4 stores
  const int Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
  bool bad = false;
#pragma unroll
  for (int wn = 0; wn < 2; ++wn) {
    const int m = m0 + wave * 64 + wn * 32 + l32;
    if (m > mlast) continue;
    const int y = m / a.W, x = m - y * a.W;
    float* op = out_f + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8;
#pragma unroll
    for (int wm = 0; wm < 2; ++wm) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = wm * 32 + 4 * h + 8 * q;
        if (co >= a.cout) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[wm][wn][4 * q + e] * a.wscale_inv + s_b[co + e];
          if (a.act == ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
          else if (a.act == ACT_PRELU) v[e] = v[e] >= 0.f ? v[e] : v[e] * s_b[RGB_BCO + co + e];
          bad |= !(__builtin_fabsf(v[e]) < 65504.f);
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
  if (bad) atomicOr(a.range_flag, 1);
}

bool x3_rgb_fits(const ConvLaunch& c) {
  return c.ks == 3 && c.cin_chunks == 1 && c.cout <= RGB_BCO && c.in_pad >= 1 && !c.hpool;
}

hipError_t launch_conv_x3_rgb(const ConvLaunch& c, hipStream_t s) {
  if (!x3_rgb_fits(c) || !c.wx3 || !c.range_flag || ((c.in_cs | c.out_cs | c.out_coff | c.in_coff) & 7)) {
    set_error("conv_x3_rgb: needs a 3x3 layer with one input chunk, <= 64 outputs and rgb-packed weights");
    return hipErrorInvalidValue;
  }
  X3Args a{};
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.wpk = (const f16x8*)c.wx3; a.bias = c.bias; a.slope = c.slope;
  a.range_flag = c.range_flag;
  a.wscale_inv = c.wscale_inv;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.cin_chunks = 1; a.pairs = 1; a.cout = c.cout;
  a.co_tiles = 1;
  // 256-pixel blocks: 3 % faster than 512 (more blocks resident per CU), 128 lost 16 %
  // (tools/archive/gpu_rgb_bpx.sh)
  constexpr int bpx = RGB_TILE;
  a.px_tiles = (c.H * c.W + bpx - 1) / bpx;
  a.tpx = bpx;
  a.act = c.act;
  a.ksplit = 1;
  a.nfr = c.n;
  const long long nb = (long long)c.n * a.px_tiles;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("conv_x3_rgb: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  t_last_variant = x3_variant_code(X3V_RGB, 3, bpx, RGB_BCO);
  hipLaunchKernelGGL(conv_x3_rgb<bpx>, dim3(a.nblocks), dim3(bpx), 0, s, a);
  return hipGetLastError();
}

double conv_x3_rgb_mfma_flops(const ConvLaunch& c) {
  return 3.0 * 2.0 * RGB_BCO * 32.0 * (double)((c.H * c.W + RGB_TILE - 1) / RGB_TILE) * RGB_TILE * c.n;
}

__global__ void __launch_bounds__(256) x3_splitk_reduce(X3Args a) {
  const int HW = a.H * a.W, c8 = (a.cout + 7) / 8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)a.nfr * c8 * HW * 2) return;
  const int h = (int)(i & 1);
  const long long q = i >> 1;
  const int m = (int)(q % HW);
  const long long r = q / HW;
  const int cc = (int)(r % c8), n = (int)(r / c8);
  x3_reduce_item(a, n, cc, m, h);
}


// ---------------------------------------------------------------------------
// Wave-range kernel (VAR 8): the small grids whose canonical K ranges would run across blocks
// (x3_ranges: fewer 128-pixel blocks than CUs -- batch-1 Mode R's 23x41 stage layers, conv4_x
// and Mconv7, the hand's 23^2 scale at small crop counts).  There the split-K form costs two
// dependent launches per layer (the range blocks, then x3_splitk_reduce reading their partial
// sums back from the workspace), and every block walks a chain of L2 round trips through LDS
// staging and barriers (~13 us per layer).
// Here one block is one output tile of 32 channels x 32 WN pixels of one frame, and wave r of
// the block sums canonical K range r (blockDim = 64 S).  A wave loads its operands straight
// into registers, DEPTH taps ahead: the pre-split weight fragments of its 32 rows (16 B per
// lane and half, the pack_x3 slab) and the 8-channel input chunk of its pixel (32 B per lane,
// split in registers by x3_split8).  No LDS staging, no barrier in the K loop.  Each wave runs
// exactly the MFMA sequence of its range in conv_x3_f16 -- (pair, ky, kx), then hi*hi, hi*lo,
// lo*hi, from zero, a missing odd chunk as zeros (the generic loop) -- the range sums meet in
// LDS and are added in x3_canonical_order, then the epilogue of x3_splitk_reduce: the same bits
// as the split-K launches and as the in-block ranges of larger batches, in one launch.
template <int KS, int WN, int DEPTH>
__global__ void __launch_bounds__(512) conv_x3_wr(X3Args a) {
  constexpr int P = KS / 2;
  constexpr int TP = KS * KS;                     // taps per chunk pair
  const int S = a.ksplit;                         // waves = K ranges
  int bid = blockIdx.x;
  {   // XCD-aware order (conv_x3_f16): the channel tiles of a pixel tile on one XCD / L2
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int co_t = bid % a.co_tiles;              // 32-channel tiles
  const int rest = bid / a.co_tiles;
  const int pt = rest % a.px_tiles;
  const int n = rest / a.px_tiles;
  const int HW = a.H * a.W;
  const int m0 = pt * 32 * WN;
  const int mlast = min(m0 + 32 * WN, HW) - 1;
  const int Wi = a.W + 2 * a.in_pad;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const float* in_f = a.in + (size_t)n * a.in_fs;
  // padded linear index of this lane's pixels at tap (ky, kx) = (0, 0)
  int Lb[WN];
#pragma unroll
  for (int wn = 0; wn < WN; ++wn) {
    const int m = min(m0 + wn * 32 + l32, mlast);
    const int y = m / a.W, x = m - y * a.W;
    Lb[wn] = (y + a.in_pad - P) * Wi + x + a.in_pad - P;
  }
  // this wave's range (conv_x3_f16 SPLIT: ceil(pairs / S) pairs per range, none empty)
  const int pps = (a.pairs + S - 1) / S;
  const int c2a = wave * pps, c2b = min(a.pairs, c2a + pps);
  const int U = (c2b - c2a) * TP;
  const int BCO = a.bco_pack, WS1 = KS * 4 * BCO;
  const int co0 = co_t * 32, cpk = co0 / BCO;
  const f16x8* wb = a.wpk + (size_t)cpk * a.pairs * KS * WS1 + h * BCO + (co0 - cpk * BCO) + l32;

  f16x8 A[DEPTH][2];
  f32x4 B[DEPTH][WN][2];
  // tap u of the range -> its operands; past the end the last tap is read again (every load
  // unconditional: the same count in flight on every path, so the waits stay counted)
  auto load = [&](int u, f16x8 (&Ad)[2], f32x4 (&Bd)[WN][2]) __attribute__((always_inline)) {
    u = min(u, U - 1);
    const int pr = u / TP, r = u - pr * TP, ky = r / KS, kx = r - ky * KS;
    const int c2 = c2a + pr;
    const f16x8* w = wb + (size_t)(c2 * KS + ky) * WS1 + kx * 4 * BCO;
    Ad[0] = w[0];
    Ad[1] = w[2 * BCO];
    const int c = min(2 * c2 + h, a.cin_chunks - 1);
    const float* src = in_f + (size_t)c * a.in_chs + (size_t)(ky * Wi + kx) * 8;
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) {
      Bd[wn][0] = *(const f32x4*)(src + (size_t)Lb[wn] * 8);
      Bd[wn][1] = *(const f32x4*)(src + (size_t)Lb[wn] * 8 + 4);
    }
  };
  f32x16 acc[WN];
#pragma unroll
  for (int wn = 0; wn < WN; ++wn)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[wn][r] = 0.f;
#ifdef ISLPOSE_DEV
  // development (tools/convbench, CONVBENCH_WRSTAMP=1): s_memtime phase stamps of wave 0 of every
  // block -- start, first operands in, K loop done, ranges combined, stores issued -- and
  // s_memrealtime at start and end (the clock)
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if (a.dbg && wave == 0 && lane == 0) {
      if (k == 0 || k == 5) a.dbg[(size_t)blockIdx.x * 8 + (k == 0 ? 6 : 7)] = __builtin_amdgcn_s_memrealtime();
      if (k < 5) a.dbg[(size_t)blockIdx.x * 8 + k] = __builtin_amdgcn_s_memtime();
    }
  };
#else
  auto stamp = [&](int) __attribute__((always_inline)) {};
#endif
  stamp(0);
  // the epilogue's bias / slopes requested before the K loop (its first group: the only one
  // when 4 WN <= S), not one memory round trip after the range sums meet
  const int co_e = min(co0 + 8 * (wave & 3) + 4 * h, a.cout - 1) & ~3;
  const f32x4 bias_e = *(const f32x4*)(a.bias + co_e);
  const f32x4 slope_e = a.act == ACT_PRELU ? *(const f32x4*)(a.slope + co_e) : f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int u, const f16x8 (&Ad)[2], const f32x4 (&Bd)[WN][2]) __attribute__((always_inline)) {
    const int pr = u / TP;
    const bool real = 2 * (c2a + pr) + h < a.cin_chunks;   // a missing odd chunk: zeros
#pragma unroll
    for (int wn = 0; wn < WN; ++wn) {
      f16x8 bh, bl;
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      x3_split8(real ? Bd[wn][0] : z, real ? Bd[wn][1] : z, bh, bl);
      acc[wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ad[0], bh, acc[wn], 0, 0, 0);
      acc[wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ad[0], bl, acc[wn], 0, 0, 0);
      acc[wn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ad[1], bh, acc[wn], 0, 0, 0);
    }
  };
  // Slot d's loads are issued in slot order (sched_barrier: the scheduler must not reorder them
  // across slots, or the wait-count pass sees a slot's registers loaded last in the prologue and
  // drains the pipeline at the loop head), so at slot d's compute DEPTH - 1 slots of loads stay
  // in flight (vmcnt((DEPTH - 1) * (2 + 2 WN)), counted by the compiler).
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) {
    load(d, A[d], B[d]);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int u0 = 0; u0 < U; u0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (u0 + d < U) compute(u0 + d, A[d], B[d]);   // (uniform)
      if (u0 == 0 && d == 0) stamp(1);
      __builtin_amdgcn_sched_barrier(0);
      load(u0 + d + DEPTH, A[d], B[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  stamp(2);
  // the ranges' sums through LDS: [range][wn][q][lane] x 4 floats (registers 4q .. 4q + 3)
  __shared__ f32x4 xch[8 * WN * 4 * 64];
#pragma unroll
  for (int wn = 0; wn < WN; ++wn)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      xch[((wave * WN + wn) * 4 + q) * 64 + lane] =
          f32x4{acc[wn][4 * q], acc[wn][4 * q + 1], acc[wn][4 * q + 2], acc[wn][4 * q + 3]};
  __syncthreads();
  stamp(3);
  // x3_canonical_order over the (wn, q) groups, spread over the waves; then x3_splitk_reduce's
  // epilogue
  const int hh = (S + 1) / 2, Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
  bool bad = false;
  for (int g = wave; g < WN * 4; g += S) {
    const int wn = g >> 2, q = g & 3;
    const int m = m0 + wn * 32 + l32;
    const int co = co0 + 8 * q + 4 * h;
    f32x4 lo = f32x4{0.f, 0.f, 0.f, 0.f}, hi = lo;   // onto +0, as the in-block sums
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= S) break;
      const f32x4 v = xch[((k * WN + wn) * 4 + q) * 64 + lane];
      if (k < hh) lo += v;
      else hi += v;
    }
    const f32x4 sum = S > hh ? lo + hi : lo;
    if (m > mlast || co >= a.cout) continue;
    const bool first = g == wave;               // the group whose operands were prefetched
    const f32x4 b = first ? bias_e : *(const f32x4*)(a.bias + co);
    const f32x4 sl = first ? slope_e : a.act == ACT_PRELU ? *(const f32x4*)(a.slope + co) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = sum[e] * a.wscale_inv + b[e];
    if (a.act == ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    } else if (a.act == ACT_PRELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) bad |= co + e < a.cout && !(__builtin_fabsf(v[e]) < 65504.f);
    const int y = m / a.W, x = m - y * a.W;
    float* oc = out_f + (size_t)(co >> 3) * a.out_chs + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8 + (co & 7);
    if (co + 3 < a.cout) {
      *(f32x4*)oc = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < a.cout) oc[e] = v[e];
    }
  }
  stamp(4);
  stamp(5);
  if (bad) atomicOr(a.range_flag, 1);
}

// Tail tiles.  A chip-filling grid of full tiles takes ceil(blocks / CUs) rounds of one block per
// CU, its last round often part-empty (Mode N's 92x164 layers: 1920 blocks, 7.5 rounds -> 8; the
// layer time follows the rounds, tools/round_probe.py).  Where it pays by the estimate below, each
// frame's first full_tiles tiles fill whole rounds and the rest of its pixels run as tail tiles of
// ttpx pixels (a multiple of 128, so that the MFMA-skipping waves past the tile stay spread over
// the SIMDs), dispatched after them.  The plan prices a tail block at 0.3 + 0.7 ttpx / tpx of a
// full one; measured, a 256-pixel tail of the 512-pixel row union costs ~0.85 (its weight slabs,
// staging and barriers stay: profiles/r05/r5tl), so only clear wins are taken (>= 0.25 round by
// the estimate).  Every output keeps its MFMA sequence: same bits.
// ISLPOSE_X3_TAIL=0: one tiling (A/B; read per launch).
static int device_cus();
static void x3_tail_plan(int n, int HW, X3Args& a) {
  a.nb_full = a.full_tiles = a.tail_tiles = a.ttpx = 0;
  const char* e = getenv("ISLPOSE_X3_TAIL");
  if (e && e[0] == '0') return;
  const long long cus = device_cus(), per = (long long)n * a.co_tiles;
  const long long R0 = (per * a.px_tiles + cus - 1) / cus;
  const int full_max = HW / a.tpx;
  const long long Rf = per * full_max / cus;        // whole rounds the full tiles can fill
  if (Rf < 1 || R0 < 2) return;
  const int F = (int)(Rf * cus / per);
  const long long NF = per * F;
  if (F < 1 || NF % 8) return;                      // (each class is spread over the 8 XCDs)
  const int rem = HW - F * a.tpx;
  double best = (double)R0 - 0.25;
  for (int t = 128; t < a.tpx; t += 128) {
    const int TT = (rem + t - 1) / t;
    const long long NT = per * TT;
    const double est = (double)NF / cus + (double)((NT + cus - 1) / cus) * (0.3 + 0.7 * t / a.tpx);
    if (est < best && NF + NT <= 0x7fffffff) {
      best = est;
      a.nb_full = (int)NF; a.full_tiles = F; a.tail_tiles = TT; a.ttpx = t;
      a.nblocks = (int)(NF + NT);
    }
  }
}

template <int KS, int WAVES_M, int WAVES_N, int WM, int WN, int VAR, int OCC>
static hipError_t launch_t(const ConvLaunch& c, hipStream_t s) {
  constexpr int BCO = WAVES_M * WM * 32;
  constexpr int BPX = WAVES_N * WN * 32;
  // (the fused pair's 512-channel tile does not fit the 4-bit tile field: it records BCO / 2,
  // decode_variant doubles it back for VAR 16)
  t_last_variant = x3_variant_code(VAR, KS, BPX, (VAR & 16) ? BCO / 2 : BCO);
  constexpr int P = KS / 2;
  constexpr int SEGCAP = x3_segmax(BPX);
  constexpr bool SPLIT = (VAR & 2048) != 0, RANGED = (VAR & 1024) != 0;
  if (c.in_pad < P) { set_error("conv_x3: input ring narrower than kernel radius"); return hipErrorInvalidValue; }
  constexpr bool HALFCO = (VAR & 256) != 0;
  if (c.bco != (HALFCO ? 2 * BCO : BCO)) { set_error("conv_x3: tile mismatch"); return hipErrorInvalidValue; }
  if ((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) { set_error("conv_x3: slice not on a chunk"); return hipErrorInvalidValue; }
  if (!c.wx3 || !c.range_flag) { set_error("conv_x3: split weights / range flag missing"); return hipErrorInvalidValue; }
  if ((SPLIT || RANGED) && c.ksplit < 2) { set_error("conv_x3: K ranges without a range count"); return hipErrorInvalidValue; }
  if (SPLIT && !c.ws) { set_error("conv_x3: split-K without workspace"); return hipErrorInvalidValue; }
  if ((VAR & 16384) && !c.dbg) { set_error("conv_x3: stamp build without a stamp buffer"); return hipErrorInvalidValue; }
  if ((VAR & 4096) && ((c.cin_chunks + 1) / 2) % 2) { set_error("conv_x3: two pairs per step needs an even pair count"); return hipErrorInvalidValue; }
  X3Args a{};
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  if (c.vin) {   // the pool's pair-max buffer: [n][chunk][2H][W][8], unpadded
    if (c.in_coff) { set_error("conv_x3: pooled-input staging reads whole buffers"); return hipErrorInvalidValue; }
    if ((long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) >= (1 << 20)) {
      set_error("conv_x3: pooled-input plane too large for the staging index math");
      return hipErrorInvalidValue;
    }
    // the pair-max buffer must be exactly 2H x W (even pre-pool height): the chunk stride
    // below assumes it (runtime pool_into_next_conv checks the producer's height)
    a.in_chs = (long long)2 * c.H * c.W * 8;
  }
  a.vin = c.vin;
  a.fold = c.fold;
  if ((VAR & 16) != 0) {
    if (c.cout7 <= 0 || c.cout7 > 64 || !c.wx3f7 || !c.bias7 || (c.act7 == ACT_PRELU && !c.slope7) || c.cout != BCO ||
        c.hpool || c.vin || c.fold || c.fold_out || c.ksplit > 1) {
      set_error("conv_x3: fused 1x1 pair needs Mconv7 filters, <= 64 outputs and one tile of every Mconv6 channel");
      return hipErrorInvalidValue;
    }
    a.wpk7 = (const f16x8*)c.wx3f7;
    a.bias7 = c.bias7;
    a.slope7 = c.slope7;
    a.wscale7_inv = c.wscale7_inv;
    a.cout7 = c.cout7;
    a.act7 = c.act7;
  } else if (c.cout7 > 0) {
    set_error("conv_x3: fused-pair launch on a plain variant");
    return hipErrorInvalidValue;
  }
#ifdef ISLPOSE_DEV
  a.abl = getenv("ISLPOSE_X3_ABL") ? atoi(getenv("ISLPOSE_X3_ABL")) : 0;
#else
  a.abl = 0;
#endif
  if ((c.fold != nullptr) != ((VAR & 8192) != 0)) { set_error("conv_x3: fold variant mismatch"); return hipErrorInvalidValue; }
  if (c.vin != ((VAR & 32768) != 0)) { set_error("conv_x3: pooled-input variant mismatch"); return hipErrorInvalidValue; }
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.wpk = (const f16x8*)c.wx3; a.bias = c.bias; a.slope = c.slope;
  a.range_flag = c.range_flag;
  a.wscale_inv = c.wscale_inv;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.cin_chunks = c.cin_chunks; a.pairs = (c.cin_chunks + 1) / 2; a.cout = c.cout;
  a.co_tiles = HALFCO ? 2 * ((c.cout + 2 * BCO - 1) / (2 * BCO)) : (c.cout + BCO - 1) / BCO;
  a.tpx = tile_pixels(c, BPX, SEGCAP);
  if (c.hpool && (a.tpx & 1)) --a.tpx;          // pair-max epilogue: tiles start on even pixels
  a.px_tiles = (c.H * c.W + a.tpx - 1) / a.tpx;
  a.act = c.act;
  a.ksplit = (SPLIT || RANGED) ? c.ksplit : 1;
  a.nfr = c.n;
  a.ws = c.ws;
  a.dbg = c.dbg;
  a.hpool = c.hpool;
  if (c.hpool) {
    if ((c.W & 1) || c.out_pad || c.out_coff || SPLIT) {
      set_error("conv_x3: pair-max epilogue needs an even width, an unpadded output and no split-K");
      return hipErrorInvalidValue;
    }
    a.out_chs = (long long)c.H * (c.W / 2) * 8;
    a.out_fs = a.out_chs * (c.out_cs / 8);
    a.out = c.out;
  }
  const long long nb = (long long)c.n * a.px_tiles * a.co_tiles * (SPLIT ? a.ksplit : 1);
  if (nb <= 0 || nb > 0x7fffffff) { set_error("conv_x3: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  if constexpr (!SPLIT && !RANGED && !(VAR & 16) && BPX >= 256) x3_tail_plan(c.n, c.H * c.W, a);
  hipLaunchKernelGGL((conv_x3_f16<KS, WAVES_M, WAVES_N, WM, WN, VAR, OCC>), dim3(a.nblocks),
                     dim3(WAVES_M * WAVES_N * 64 * ((VAR & 32) ? 2 : 1)), 0, s, a);
  if constexpr (SPLIT) {
    // fold_out: every consumer sums the partials in its staging (X3Fold), no reduce launch
    if (!c.fold_out) {
      const long long nt = (long long)c.n * ((c.cout + 7) / 8) * 2 * c.H * c.W;
      hipLaunchKernelGGL(x3_splitk_reduce, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, a);
    }
  } else {
    if (c.fold_out) { set_error("conv_x3: fold_out without split-K across blocks"); return hipErrorInvalidValue; }
  }
  return hipGetLastError();
}

static bool x3_small_tiles() {
  static const bool v = getenv("ISLPOSE_X3_TILES") && getenv("ISLPOSE_X3_TILES")[0] == 's';
  return v;
}

// 0: no row union (A/B), 1: row union (default), 4: row union with s_memtime stamps
// (development; needs ConvLaunch::dbg, set only by tools/convbench)
static int x3_union_mode() {
  static const int m = getenv("ISLPOSE_X3_UNION") ? atoi(getenv("ISLPOSE_X3_UNION")) : 1;
  return m;
}

static int device_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return cus > 0 ? cus : 256;
  }();
  return n;
}

// Canonical K ranges of a layer, from its shape alone (never the batch): the small
// stage layers (<= 1024 pixels per frame: Mode R's 23x41 body stages, the 184 px hand
// scale) sum their chunk pairs in S ranges, so that a batch-1 frame can spread them
// over S blocks (split-K) and a large batch can keep them in one block, with the same
// bits.  Every range is ceil(pairs / S) pairs long and non-empty.
// Small grids (the 128-pixel family) with 128-channel tiles on two 64-channel blocks of 4
// waves each (VAR 256): by default the 1x1 / 3x3 layers whose K ranges are split across
// blocks (grids below one block per CU: batch-1 Mode R, +4 % frames/s), where doubling the
// grid buys more than the second staging of the input costs; with one block per CU (Mode R
// batch 32) it loses 10-20 % (profiles/r03/halfco_ab/).  Same bits either way.
// ISLPOSE_X3_HALFCO=0 off, =1 every 128-channel launch of the family (read per launch; A/B).
static bool x3_small7(const ConvLaunch& c);
static bool x3_halfco(const ConvLaunch& c) {
  if (c.ks > 7 || c.fold) return false;
  if (c.ks == 7) return c.ksplit > 1 && c.ws && x3_small7(c);
#ifdef ISLPOSE_DEV
  // development build only (A/B of profiles/r03/halfco_ab/): =0 off, =1 every 128-channel
  // launch of the family (measured slower at one block per CU, so not in the product)
  const char* e = getenv("ISLPOSE_X3_HALFCO");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
#endif
  return c.ks <= 3 && c.ksplit > 1 && c.ws;
}

// Small 7x7 grids (a frame's hand crops per call: one or two crops at the 46^2 - 92^2 hand
// scales, or the 23^2 scale's across-block K ranges), under one 128-pixel block per CU: the
// 128-channel tiles run as two 64-channel blocks on 64-pixel tiles (VAR 256, 4 waves of 32co x
// 32px, two blocks per CU): 4x the blocks, each output the same MFMA sequence (same ranges, same
// K order), so the same bits as the batched crops.  ISLPOSE_X3_SMALL7=0 off (A/B; per launch).
static int x3_small7_mode() {
  const char* e = getenv("ISLPOSE_X3_SMALL7");
  return e ? atoi(e) : 2;
}
static bool x3_small7(const ConvLaunch& c) {
  if (c.ks != 7 || c.bco != 128 || c.fold || c.vin || c.hpool) return false;
  if (x3_small7_mode() == 0) return false;
  const int tpx = tile_pixels(c, 128, x3_segmax(128));
  const long long blocks = (long long)c.n * ((c.H * c.W + tpx - 1) / tpx) * std::max(1, c.ksplit);
  return blocks < device_cus();
}
// ... with the operands two K steps ahead (VAR 128: a ring of three 28 KiB weight slabs, one
// block per CU) where the 64-pixel grid still fits one block per CU: the 46^2 / 69^2 scales
// of one crop 55 -> 48 us per layer; past one round (92^2: 266 blocks) the two resident
// blocks of the plain loop win (profiles/r05/r5s7b/).  ISLPOSE_X3_SMALL7=1: never, 3: always.
static bool x3_small7_deep(const ConvLaunch& c) {
  const int m = x3_small7_mode();
  if (m < 2) return false;
  if (m >= 3) return true;
  const int tpx = tile_pixels(c, 64, x3_segmax(64));
  return (long long)c.n * ((c.H * c.W + tpx - 1) / tpx) * 2 * std::max(1, c.ksplit) <= device_cus();
}

// ... on 96-pixel tiles (6 waves of 32co x 32px, two steps ahead) where the 64-pixel grid takes
// more than one round of one block per CU and the 96-pixel grid takes one: one crop at the
// 92^2 (736 px) hand scale, 266 -> 178 blocks (the 64-pixel plain loop left 10 CUs with two
// blocks, every layer waiting on them).  No K range is split: the same bits.
// ISLPOSE_X3_S7W96=0 off (A/B; read per launch).
static bool x3_small7_96(const ConvLaunch& c) {
  const char* e = getenv("ISLPOSE_X3_S7W96");
  if ((e && e[0] == '0') || x3_small7_mode() != 2 || c.ksplit > 1) return false;
  const long long HW = (long long)c.H * c.W, cus = device_cus();
  const int t64 = tile_pixels(c, 64, x3_segmax(64)), t96 = tile_pixels(c, 96, x3_segmax(96));
  return c.n * ((HW + t64 - 1) / t64) * 2 > cus && c.n * ((HW + t96 - 1) / t96) * 2 <= cus;
}

// Small grids (the 128-pixel family) with two K groups per block (VAR 32, 16 waves: the first
// and second half of the canonical K ranges side by side, one block per CU): every 128-channel
// 1x1 / 3x3 launch whose K ranges run in one block (Mode R's 23x41 stage layers and conv4_x at
// batch >= 32; 5-6 % faster than the one-group loops there, profiles/r04/r4b/).  The 96-channel
// form (two groups of 6 waves of 32co x 64px) measured 7 % slower than the deep-prefetch loop on
// the c96 stage layers and is not built.  The one-group form keeps both halves' sums and the
// range's in registers (153 VGPRs: one 8-wave block per CU) where two groups hold one each (122:
// 16 waves per CU).
// ISLPOSE_X3_G2=0: the one-group loops (A/B; read per launch).
static bool x3_g2(const ConvLaunch& c) {
  if (c.ks > 3 || c.bco != 128 || c.fold || c.vin || c.ksplit < 2 || c.ws) return false;
  const char* e = getenv("ISLPOSE_X3_G2");
  return !(e && e[0] == '0');
}

// Small grids whose K ranges run across blocks (batch-1 Mode R's 23x41 stage layers: 8 pixel
// tiles x S ranges, far under one block per CU) on 64-pixel tiles: the 96-channel tiles as 6
// waves of 32co x 32px (not 12 on 128 pixels), the half-channel blocks of the 128-channel tiles
// (VAR 256) as 4 waves of 32co x 32px (not 4 of 64co x 32px on 128 pixels) -- twice the blocks,
// each with half the MFMAs and staging per K step.  Each output sees the same MFMA sequence (same
// ranges, same K order): same bits.  Batch-1 Mode R net 1.955 -> 1.828 ms (profiles/r04/r4ai/).
// ISLPOSE_X3_PX64=0: the 128-pixel blocks, =1: the 96-channel tiles only (A/B; read per launch).
static int x3_px64_mode() {
  const char* e = getenv("ISLPOSE_X3_PX64");
  return e ? atoi(e) : 2;
}
static bool x3_px64(const ConvLaunch& c) {
  if (c.ks > 3 || c.bco != 96 || c.fold || c.vin || c.ksplit < 2 || !c.ws) return false;
  return x3_px64_mode() >= 1;
}

// Small 3x3 grids without K ranges (batch-1 conv2_x / conv3_x: at most half a block per CU) on
// half-channel blocks (VAR 256): twice the blocks; same MFMA sequence per output, same bits.
// Batch-1 Mode R net 1.828 -> 1.817 ms; the 1x1 layers (the two-launch Mconv6) measured slower
// and the deep-prefetch form level (profiles/r04/r4ai/).  ISLPOSE_X3_HALFSMALL=0 off (A/B).
static bool x3_halfsmall(const ConvLaunch& c) {
  const char* e = getenv("ISLPOSE_X3_HALFSMALL");
  if ((e && e[0] == '0') || c.ks != 3 || c.bco != 128 || c.fold || c.vin || c.ksplit > 1) return false;
  const int tpx = tile_pixels(c, 128, x3_segmax(128));
  const long long blocks = (long long)c.n * ((c.H * c.W + tpx - 1) / tpx) * ((c.cout + c.bco - 1) / c.bco);
  return 2 * blocks <= device_cus();
}

// Small grids (the 128-pixel family) with the inputs and weights prefetched two K steps
// ahead (VAR 128): by default the 3x3 layers whose grid has at most one block per CU and
// whose K ranges (if any) run in one block -- Mode R's 23x41 stage layers at batch 32, -5 to
// -12 % per layer in the net (profiles/r03/deep_ab/).  Its ring of three weight slabs (98 KiB)
// allows one block per CU, so grids with more blocks lose the second resident block (conv4_x
// at batch 32: +12-16 %), and the 1x1 layers lost 25-30 %.  ISLPOSE_X3_DEEP=0 off, =1 every
// 1x1 / 3x3 launch of the family, across-block ranges included (A/B; read per launch).
static bool x3_deep(const ConvLaunch& c) {
  const char* e = getenv("ISLPOSE_X3_DEEP");
  if (c.fold || c.vin || (c.bco != 128 && c.bco != 96) || c.ks > 3) return false;
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  if (c.ks != 3 || (c.ksplit > 1 && c.ws)) return false;
  const int tpx = tile_pixels(c, 128, x3_segmax(128));
  const long long blocks = (long long)c.n * ((c.H * c.W + tpx - 1) / tpx) * ((c.cout + c.bco - 1) / c.bco);
  return blocks <= device_cus();
}

// Small grids (the 128-pixel family) with two chunk pairs per K step (VAR 4096): a step's
// MFMAs double against its barrier and its L2 round trip.  Only for layers with canonical K
// ranges (they never run the big-tile kernels, whose one-pair order the other layers must
// keep for batch-invariant bits), an even number of pairs in every range, and one channel
// tile (c512 lost 7 %).  Per layer (tools/convbench, 23x41 at batch 32) c128 -3 %, c96 -8 %,
// c384 / c288 -1.5 % time, but the whole of Mode R moved by +-1 % (batch 32 +0.5 %, batch 1
// -1.2 %, profiles/r03/pps2_ab/), so it is off by default.  ISLPOSE_X3_PPS2=1: on (A/B; read
// per launch).
static int x3_canonical_ranges(const ConvLaunch& c);
#ifdef ISLPOSE_DEV
static bool x3_pps2(const ConvLaunch& c) {
  // the fold A/B (ISLPOSE_X3_FOLD=1) runs its consumers on one-pair steps, so every layer of a
  // frame keeps one order at every batch size only with PPS2 off there
  const char* e = getenv("ISLPOSE_X3_PPS2");
  const char* f = getenv("ISLPOSE_X3_FOLD");
  if (!(e && e[0] == '1') || (f && f[0] == '1') || c.ks > 3 || c.vin || (c.bco != 128 && c.bco != 96) ||
      c.cout > c.bco)
    return false;
  const int S = x3_canonical_ranges(c), pairs = (c.cin_chunks + 1) / 2;
  if (S < 2 || c.ksplit != S) return false;
  const int pps = (pairs + S - 1) / S;
  return pairs % 2 == 0 && pps % 2 == 0;
}
#else
static bool x3_pps2(const ConvLaunch&) { return false; }   // rejected (profiles/r03/pps2_ab/): dev build only
#endif

static int x3_canonical_ranges(const ConvLaunch& c) {
  // 3x3 / 7x7 layers: ranges of >= 2 chunk pairs; 1x1 layers: >= 4 pairs (64 channels), so
  // that a range of an Mconv7 is one wave's share of the fused pair (VAR 16) and the two
  // executions of the pair give the same bits
  const int pairs = (c.cin_chunks + 1) / 2, per = c.ks == 1 ? 4 : 2;
  if (!c.allow_split || c.H * c.W > 1024 || pairs < 2 * per) return 1;
  int S = std::min(8, pairs / per);
  while (S > 1 && (S - 1) * ((pairs + S - 1) / S) >= pairs) --S;
  return S;
}

// Tile families.  3x3 / 1x1 layers: 512-pixel tiles (16 waves per block, one
// block per CU): the weight slab of a K step is then shared by 4x the pixels,
// which cut the L2->LDS bytes per FLOP ~2x and measured +10 % over the 128-pixel
// tiles (r01); 16 rather than 8 waves for the narrow (96/64/32-channel) tiles
// +2-9 %.  7x7 layers keep 128-pixel tiles (their slab is 2.3x larger), and so do
// layers with canonical K ranges (their second accumulator set needs the 128-pixel
// family's register budget).  512-pixel tiles are used only when they fill the
// chip: a layer with fewer such blocks than CUs runs ~2x faster on the 128-pixel,
// 4-wave family (tools/archive/gpu_tiles.sh).
static bool x3_union(const ConvLaunch& c);

// 64-channel 3x3 layers off the row union (full-resolution conv1_2 / hand conv1_2: 12 K
// steps) run 256-pixel blocks of 8 waves (64co x 32px each), two blocks per CU, so that one
// block's prologue and epilogue overlap the other's K loop: -4 to -5 % against the 16-wave
// 512-pixel block (tools/archive/gpu_mid.sh; the 128-channel layers stay on 512 pixels, where every
// 256-pixel shape lost 4-7 %).  ISLPOSE_X3_HALF64=0: the 512-pixel block (A/B).
static bool x3_half64(const ConvLaunch& c) {
  static const bool on = !(getenv("ISLPOSE_X3_HALF64") && getenv("ISLPOSE_X3_HALF64")[0] == '0');
  return on && c.ks == 3 && c.bco == 64 && !x3_union(c);
}

static int x3_big_bpx(const ConvLaunch& c) { return (c.ks == 1 && c.bco == 256) || x3_half64(c) ? 256 : 512; }

static bool x3_big_tiles(const ConvLaunch& c) {
  if (c.ks > 3 || x3_small_tiles() || x3_canonical_ranges(c) > 1) return false;
  const int bpx = x3_big_bpx(c), tpx = tile_pixels(c, bpx, x3_segmax(bpx));
  const long long px_tiles = (c.H * c.W + tpx - 1) / tpx;
  return (long long)c.n * px_tiles * ((c.cout + c.bco - 1) / c.bco) >= device_cus();
}

// 1x1 layers with 256k output channels and an even number of chunk pairs (Mconv6 of
// every stage: 384/288 -> 512/256) also pack their split filters for 256-channel
// tiles.  On big grids they run 16 waves of 64co x 64px over 256 pixels with two chunk
// pairs per K step (VAR 4096: 24 MFMAs per wave between barriers instead of 12, and
// the input read for half as many channel tiles): +7-12 % (tools/archive/gpu_k1.sh).  Small
// grids (K ranges, the 128-pixel family) keep the 128-channel packing: 256-channel
// tiles there halve the blocks and lost 30 %.
bool x3_wide1_layer(int ks, int cout, int cin_phys) {
  return ks == 1 && cout % 256 == 0 && ((cin_phys / 8 + 1) / 2) % 2 == 0;
}

bool x3_wide1(const ConvLaunch& c) {
  return c.bco == 256 && x3_wide1_layer(c.ks, c.cout, c.cin_chunks * 8) && x3_big_tiles(c);
}

// 7x7 layers on 256-pixel tiles (8 waves of 64co x 64px, 156 KiB of LDS) or on
// 128-pixel tiles (8 waves of 64co x 32px): one block per CU either way (a step's
// weight slab is 56 KiB).  The 256-pixel block does twice the work for ~1.72x the
// time of a 128-pixel block (half the weight bytes per MFMA), so the choice is per
// launch, by grid quantisation: rounds of one block per CU, a 256-pixel block costing
// X3_WIDE7_COST 128-pixel blocks.  Both pack the weights for 128-channel tiles.
// Round 6 re-measured the three forms on the hand's batch-32 grids of C3 (op tables,
// profiles/r06/w7ab/): 69^2 x 32 ran 11.93 / 10.89 / 11.36 ms over its twenty 7x7 stage
// layers on 128 / 256 / 384 pixels (5 / 3 / 2 rounds), i.e. 1.52 and 2.38 128-pixel rounds
// per round; with the round-2 costs (1.74, 2.58; tools/archive/gpu_wide7.sh, gpu_w384.sh)
// the estimate kept 69^2 on 128 pixels.  92^2 (384) and 46^2 (384) choose as before.
constexpr double X3_WIDE7_COST = 1.52;
// a round of 384-pixel blocks (12 waves, one input buffer)
constexpr double X3_W384_COST = 2.38;

static int x3_wide7_mode() {   // ISLPOSE_X3_WIDE7: 0 never, 1 always (A/B), default by the estimate
  static const int m = getenv("ISLPOSE_X3_WIDE7") ? atoi(getenv("ISLPOSE_X3_WIDE7")) : 2;
  return m;
}

// pixels per 7x7 tile (128, 256 or 384), chosen per launch by grid quantisation: rounds
// of one block per CU, a round of 256- / 384-pixel blocks costing X3_WIDE7_COST /
// X3_W384_COST of a 128-pixel round.  ISLPOSE_X3_WIDE7=0|1|3 forces 128 / 256 / 384 (A/B).
static int x3_7x7_bpx(const ConvLaunch& c) {
  if (c.ks != 7 || c.bco != 128 || x3_small_tiles() || x3_canonical_ranges(c) > 1) return 128;
  const int mode = x3_wide7_mode();
  if (mode != 2) return mode == 1 ? 256 : mode == 3 ? 384 : 128;
  const long long HW = (long long)c.H * c.W, co = (c.cout + 127) / 128, cus = device_cus();
  int best = 128;
  double best_t = 0.0;
  for (int bpx : {128, 256, 384}) {
    const int t = tile_pixels(c, bpx, x3_segmax(bpx));
    const long long b = c.n * ((HW + t - 1) / t) * co;
    const double cost = bpx == 128 ? 1.0 : bpx == 256 ? X3_WIDE7_COST : X3_W384_COST;
    const double tt = (double)((b + cus - 1) / cus) * cost;
    if (bpx == 128 || tt < best_t) { best = bpx; best_t = tt; }
  }
  return best;
}

static bool x3_wide7(const ConvLaunch& c) { return x3_7x7_bpx(c) == 256; }

// 7x7 on 384-pixel tiles (VAR 65536, one input buffer)
static bool x3_wide7_384(const ConvLaunch& c) { return x3_7x7_bpx(c) == 384; }

// Row-union staging (VAR 512) when the longest union run of any 512-pixel tile fits.
// longest row-union run (pixels) over the 512-pixel tiles of a layer
static int x3_union_run(const ConvLaunch& c) {
  const int P = c.ks / 2, Wi = c.W + 2 * c.in_pad, HW = c.H * c.W;
  const int tpx = tile_pixels(c, 512, x3_segmax(512));
  int span = 0;
  for (int m0 = 0; m0 < HW; m0 += tpx) {
    const int ml = std::min(m0 + tpx, HW) - 1;
    span = std::max(span, (ml / c.W - m0 / c.W) * Wi + (ml % c.W - m0 % c.W));
  }
  return span + 2 * P * Wi + 2 * P + 1;
}

static bool x3_union(const ConvLaunch& c) {
  if (x3_union_mode() == 0 || c.ks != 3 || x3_small_tiles() || x3_canonical_ranges(c) > 1) return false;
  return x3_union_run(c) <= x3_segu_max();
}

// The row union on v_mfma_f32_16x16x32_f16 (VAR 131072) for 128-channel tiles with an even
// number of chunk pairs.  ISLPOSE_X3_M16=0|1 (read per launch: A/B in one process).
#ifdef ISLPOSE_DEV
static bool x3_m16(const ConvLaunch& c) {
  const char* e = getenv("ISLPOSE_X3_M16");
  const bool on = e && e[0] == '1';
  return on && c.ks == 3 && c.bco == 128 && ((c.cin_chunks + 1) / 2) % 2 == 0;
}
#else
static bool x3_m16(const ConvLaunch&) { return false; }    // rejected (profiles/r03/m16_ab/): dev build only
#endif

// K-range plan of a launch on the 128-pixel family: S ranges, computed across S blocks
// per tile (split-K, partials through the workspace) when the plain grid has fewer
// blocks than CUs, else in one block (tools/archive/gpu_across.sh: across wins 10-50 % at
// 64-160 blocks, in-block wins 20-70 % at 256-1024 -- same bits either way).  With isl_net_set_split_k(net, 2) (latency
// mode) layers without canonical ranges also split when their grid is that small --
// an adaptive S that depends on the batch, so those layers' bits then do too.
struct X3Ranges {
  int S = 1;
  bool across_blocks = false;
};

static X3Ranges x3_ranges(const ConvLaunch& c) {
  X3Ranges r;
  if (x3_big_tiles(c) || x3_7x7_bpx(c) != 128) return r;
  const int tpx = tile_pixels(c, 128, x3_segmax(128));
  const long long blocks = (long long)c.n * ((c.H * c.W + tpx - 1) / tpx) * ((c.cout + c.bco - 1) / c.bco);
  const int cus = device_cus(), pairs = (c.cin_chunks + 1) / 2;
  r.S = x3_canonical_ranges(c);
  if (r.S > 1) {
    static const int force = getenv("ISLPOSE_X3_ACROSS") ? atoi(getenv("ISLPOSE_X3_ACROSS")) : -1;   // A/B
    r.across_blocks = force >= 0 ? force == 1 : blocks < cus;
    return r;
  }
  if (c.allow_split == 2 && 2 * blocks <= cus && pairs >= 4) {
    int S = (int)std::min<long long>({8, pairs / 2, (cus + blocks - 1) / blocks});
    while (S > 1 && (S - 1) * ((pairs + S - 1) / S) >= pairs) --S;
    r.S = S;
    r.across_blocks = S > 1;
  }
  return r;
}

template <int KS>
static hipError_t launch_ks(const ConvLaunch& c, hipStream_t s) {
  if constexpr (KS == 3) {
    if (x3_big_tiles(c) && x3_union(c)) {
#ifdef ISLPOSE_DEV
      if (x3_union_mode() == 4 && c.dbg) {   // development build only (tools/convbench)
        switch (c.bco) {
          case 128: return launch_t<KS, 2, 8, 2, 2, 512 | 16384, 4>(c, s);
          case 96: return launch_t<KS, 1, 16, 3, 1, 512 | 16384, 4>(c, s);
        }
      }
#endif
#ifdef ISLPOSE_DEV
      const bool m16 = c.bco == 128 && x3_m16(c);
      if (m16) {
        if (c.vin) return launch_t<KS, 2, 8, 2, 2, 512 | 32768 | 131072, 4>(c, s);
        return launch_t<KS, 2, 8, 2, 2, 512 | 131072, 4>(c, s);
      }
#endif
      if (c.vin) {
        if (c.bco == 128) return launch_t<KS, 2, 8, 2, 2, 512 | 32768, 4>(c, s);
        set_error("conv_x3: pooled-input staging without a variant (x3_vin_ok)");
        return hipErrorInvalidValue;
      }
      switch (c.bco) {
        case 128: return launch_t<KS, 2, 8, 2, 2, 512, 4>(c, s);
        case 96: return launch_t<KS, 1, 16, 3, 1, 512, 4>(c, s);
        case 64: return launch_t<KS, 2, 8, 1, 2, 512, 4>(c, s);
        case 32: return launch_t<KS, 1, 16, 1, 1, 512, 4>(c, s);
      }
    }
  }
  if constexpr (KS == 1) {
    if (c.bco == 256 && x3_big_tiles(c)) return launch_t<KS, 4, 4, 2, 2, 4096, 1>(c, s);
  }
  if constexpr (KS <= 3) {
    if (x3_big_tiles(c)) {
      if constexpr (KS == 3) {
        if (c.vin) {
          if (c.bco == 128) return launch_t<KS, 2, 8, 2, 2, 32768, 4>(c, s);
          if (x3_half64(c)) return launch_t<KS, 1, 8, 2, 1, 32768, 2>(c, s);
        }
      }
      if (c.vin) {
        set_error("conv_x3: pooled-input staging without a variant (x3_vin_ok)");
        return hipErrorInvalidValue;
      }
      if (x3_half64(c)) return launch_t<KS, 1, 8, 2, 1, 0, 2>(c, s);   // 8 waves of 64co x 32px, 256 px
      switch (c.bco) {
        case 128: return launch_t<KS, 2, 8, 2, 2, 0, 4>(c, s);   // 16 waves, 64co x 64px each
        case 96: return launch_t<KS, 1, 16, 3, 1, 0, 4>(c, s);   // 16 waves, 96co x 32px
        case 64: return launch_t<KS, 2, 8, 1, 2, 0, 4>(c, s);    // 16 waves, 32co x 64px
        case 32: return launch_t<KS, 1, 16, 1, 1, 0, 4>(c, s);   // 16 waves, 32co x 32px
      }
    }
  }
  if constexpr (KS == 7) {
    // 128-channel 7x7 tiles without K ranges: 8 waves of 64co x 64px on 256 pixels, or
    // of 64co x 32px on 128 pixels (one block per CU either way: the 56 KiB weight
    // slabs; 8 waves measured 2-6 % over 4 waves of 64co x 64px / x 128px)
    if (c.ksplit <= 1 && c.bco == 128) {
      if (x3_small7(c)) {   // 64co x 64px blocks (=2: the steps' operands two steps ahead)
        if (x3_small7_96(c)) return launch_t<KS, 2, 3, 1, 1, 256 | 128, 1>(c, s);
        if (x3_small7_deep(c)) return launch_t<KS, 2, 2, 1, 1, 256 | 128, 1>(c, s);
        return launch_t<KS, 2, 2, 1, 1, 256, 4>(c, s);
      }
      if (x3_wide7_384(c)) return launch_t<KS, 2, 6, 2, 2, 65536, 1>(c, s);   // 12 waves, 384 px
      if (x3_wide7(c)) return launch_t<KS, 2, 4, 2, 2, 0, 1>(c, s);
      return launch_t<KS, 2, 4, 2, 1, 0, 1>(c, s);
    }
  }
  const bool ranged = c.ksplit > 1 && !c.ws;      // launch_conv_x3: in-block ranges
  const bool split = c.ksplit > 1 && c.ws;        // across blocks
  // 128- / 96-channel tiles of the 128-pixel family: 8 waves of 64co x 32px / 12 waves of
  // 32co x 32px rather than 4 waves of 64co x 64px / 96co x 32px.  These grids are small
  // (Mode R's 23x41 stages: one block per CU at batch 32), and two or three waves per
  // SIMD hide the staging: -8 to -22 % on the 23x41 3x3 stage layers, -12 to -31 % on
  // their 1x1 layers, -5 to -14 % on the hand's 23^2 7x7 layers, -20 % on its 23^2 c512
  // layers (tools/archive/gpu_s8.sh, gpu_s8b.sh).  ISLPOSE_X3_S8=0: the 4-wave layouts (A/B).
  static const int more = getenv("ISLPOSE_X3_S8") ? atoi(getenv("ISLPOSE_X3_S8")) : 1;
  if (more) {
    {
#ifdef ISLPOSE_DEV
      if constexpr (KS <= 3) {
        if (c.fold) {   // consumers of folded split-K partials (x3_fold_ok)
          switch (c.bco) {
            case 128:
              if (split) return launch_t<KS, 2, 4, 2, 1, 2048 | 8192, 2>(c, s);
              if (ranged) return launch_t<KS, 2, 4, 2, 1, 1024 | 8192, 2>(c, s);
              return launch_t<KS, 2, 4, 2, 1, 8192, 2>(c, s);
            case 96:
              if (split) return launch_t<KS, 3, 4, 1, 1, 2048 | 8192, 2>(c, s);
              if (ranged) return launch_t<KS, 3, 4, 1, 1, 1024 | 8192, 2>(c, s);
              return launch_t<KS, 3, 4, 1, 1, 8192, 2>(c, s);
          }
          set_error("conv_x3: fold without a variant (x3_fold_ok)");
          return hipErrorInvalidValue;
        }
      }
#else
      if (c.fold) {
        set_error("conv_x3: the split-K fold is a development-build variant");
        return hipErrorInvalidValue;
      }
#endif
      if constexpr (KS <= 3) {
        if (x3_g2(c)) return launch_t<KS, 2, 4, 2, 1, 1024 | 32, 1>(c, s);   // two K groups of 8 waves
      }
      if constexpr (KS <= 3) {
        if (!split && !ranged && x3_halfsmall(c)) return launch_t<KS, 1, 4, 2, 1, 256, 4>(c, s);
      }
      if constexpr (KS <= 3) {
        if (x3_deep(c)) {   // prefetch two K steps ahead
          switch (c.bco) {
            case 128:
              if (split) return launch_t<KS, 2, 4, 2, 1, 2048 | 128, 1>(c, s);
              if (ranged) return launch_t<KS, 2, 4, 2, 1, 1024 | 128, 1>(c, s);
              return launch_t<KS, 2, 4, 2, 1, 128, 1>(c, s);
            case 96:
              if (split) return launch_t<KS, 3, 4, 1, 1, 2048 | 128, 1>(c, s);
              if (ranged) return launch_t<KS, 3, 4, 1, 1, 1024 | 128, 1>(c, s);
              return launch_t<KS, 3, 4, 1, 1, 128, 1>(c, s);
          }
        }
      }
#ifdef ISLPOSE_DEV
      if constexpr (KS <= 3) {
        if (x3_pps2(c)) {   // two chunk pairs per K step: twice the MFMAs between barriers
          switch (c.bco) {
            case 128:
              if (split) return launch_t<KS, 2, 4, 2, 1, 2048 | 4096, 2>(c, s);
              if (ranged) return launch_t<KS, 2, 4, 2, 1, 1024 | 4096, 2>(c, s);
              return launch_t<KS, 2, 4, 2, 1, 4096, 2>(c, s);
            case 96:
              if (split) return launch_t<KS, 3, 4, 1, 1, 2048 | 4096, 2>(c, s);
              if (ranged) return launch_t<KS, 3, 4, 1, 1, 1024 | 4096, 2>(c, s);
              return launch_t<KS, 3, 4, 1, 1, 4096, 2>(c, s);
          }
        }
      }
#endif
      if (c.bco == 128 && x3_halfco(c)) {   // two blocks of 4 waves (64co x 32px) per 128-channel tile
        if constexpr (KS == 7) {
          if (split && x3_small7_deep(c)) return launch_t<KS, 2, 2, 1, 1, 2048 | 256 | 128, 1>(c, s);
        }
        if (split && x3_px64_mode() >= 2) return launch_t<KS, 2, 2, 1, 1, 2048 | 256, 4>(c, s);
        if (split) return launch_t<KS, 1, 4, 2, 1, 2048 | 256, 4>(c, s);
#ifdef ISLPOSE_DEV
        if (ranged) return launch_t<KS, 1, 4, 2, 1, 1024 | 256, 4>(c, s);
#endif
        if (!ranged) return launch_t<KS, 1, 4, 2, 1, 256, 4>(c, s);
      }
      switch (c.bco) {
        case 128:   // 8 waves of 64co x 32px
          if (split) return launch_t<KS, 2, 4, 2, 1, 2048, 2>(c, s);
          if (ranged) return launch_t<KS, 2, 4, 2, 1, 1024, 2>(c, s);
          return launch_t<KS, 2, 4, 2, 1, 0, 2>(c, s);
        case 96:    // 12 waves of 32co x 32px (6 on 64-pixel tiles: x3_px64)
          if (split && x3_px64(c)) return launch_t<KS, 3, 2, 1, 1, 2048, 4>(c, s);
          if (split) return launch_t<KS, 3, 4, 1, 1, 2048, 2>(c, s);
          if (ranged) return launch_t<KS, 3, 4, 1, 1, 1024, 2>(c, s);
          return launch_t<KS, 3, 4, 1, 1, 0, 2>(c, s);
      }
    }
  }
  switch (c.bco) {
#define X3_CASE(BC, WMS, WNS, WMM, WNN)                                           \
  case BC:                                                                        \
    if (split) return launch_t<KS, WMS, WNS, WMM, WNN, 2048, 2>(c, s);            \
    if (ranged) return launch_t<KS, WMS, WNS, WMM, WNN, 1024, 2>(c, s);           \
    return launch_t<KS, WMS, WNS, WMM, WNN, 0, 2>(c, s);
    X3_CASE(128, 2, 2, 2, 2)
    X3_CASE(96, 1, 4, 3, 1)
    X3_CASE(64, 1, 4, 2, 1)
    X3_CASE(32, 1, 4, 1, 1)
#undef X3_CASE
  }
  set_error("conv_x3: unsupported tile");
  return hipErrorInvalidValue;
}

bool x3_fits(const ConvLaunch& c) { return c.in_pad >= c.ks / 2; }

// Launches with a pooled-input variant (VAR 32768): 3x3 layers on the 512-pixel family
// with 128-channel tiles (row union or generic) or the 256-pixel 64-channel blocks -- the
// layers after the body's and hand's pools at batch sizes that fill the chip.  Others
// take vpool2_kernel + the plain variant.
bool x3_vin_ok(const ConvLaunch& c) {
  return x3_fits(c) && c.ks == 3 && c.in_coff == 0 && x3_ranges(c).S == 1 && x3_big_tiles(c) &&
         (c.bco == 128 || x3_half64(c)) && (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) < (1 << 20);
}

bool x3_hpool_ok(const ConvLaunch& c) {
  return x3_fits(c) && !(c.W & 1) && !(x3_ranges(c).S > 1 && x3_ranges(c).across_blocks);
}

double conv_x3_mfma_flops(const ConvLaunch& c) {
  const int BPX = x3_big_tiles(c) ? x3_big_bpx(c) : x3_wide7_384(c) ? 384 : x3_wide7(c) ? 256 : 128;
  const double co = (double)((c.cout + c.bco - 1) / c.bco) * c.bco;
  const double px = std::ceil((double)c.H * c.W / tile_pixels(c, BPX, x3_segmax(BPX))) * BPX;
  return 3.0 * 2.0 * co * (((c.cin_chunks + 1) / 2) * 16.0) * c.ks * c.ks * px * c.n;
}

int x3_split_ranges(const ConvLaunch& c, bool* across_blocks) {
  const X3Ranges r = x3_ranges(c);
  if (across_blocks) *across_blocks = r.across_blocks;
  return r.S;
}

bool x3_fold_ok(const ConvLaunch& c) {
  static const int more = getenv("ISLPOSE_X3_S8") ? atoi(getenv("ISLPOSE_X3_S8")) : 1;
  return more && x3_fits(c) && c.ks <= 3 && !c.vin && !c.hpool && (c.bco == 128 || c.bco == 96) &&
         !x3_big_tiles(c) && (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) < (1 << 20);
}

size_t x3_splitk_ws_floats(const ConvLaunch& c) {
  const X3Ranges r = x3_ranges(c);
  return r.across_blocks ? (size_t)r.S * c.n * ((c.cout + 7) / 8) * 8 * c.H * c.W : 0;
}

bool x3_fused67_fits(int cout6, int cout7) {
  return (cout6 == 128 || cout6 == 256 || cout6 == 512) && cout7 > 0 && cout7 <= 64;
}

// The fused 1x1 pair, one tile of every Mconv6 channel: 16 waves of 64co x 64px, 8 x 2
// (512 channels, 128 pixels), 4 x 4 (256, 256) or 2 x 8 (128, 512).  No K ranges: the pair
// always runs fused, at every batch size, so a frame's bits do not depend on its batch.
static hipError_t launch_x3_fused67(ConvLaunch c, hipStream_t s) {
  if (c.ks != 1 || !x3_fused67_fits(c.cout, c.cout7)) {
    set_error("conv_x3: fused 1x1 pair outside its shapes");
    return hipErrorInvalidValue;
  }
  c.ksplit = 1;
  c.ws = nullptr;
  c.bco = c.cout;
  // (two chunk pairs per K step with one input buffer, VAR 4096 | 65536, measured level with
  // this loop in Mode N and Mode R, profiles/r04/r4c/ops_*_pps1.txt: not built)
  switch (c.cout) {
    case 512: return launch_t<1, 8, 2, 2, 2, 16, 4>(c, s);
    case 256: return launch_t<1, 4, 4, 2, 2, 16, 4>(c, s);
    case 128: return launch_t<1, 2, 8, 2, 2, 16, 4>(c, s);
  }
  set_error("conv_x3: fused 1x1 pair outside its shapes");
  return hipErrorInvalidValue;
}

// The pair runs fused where its grid has at least half a block per CU; smaller grids (batch-1
// Mode R: 8 pixel tiles) take the two launches (Mconv6 then Mconv7 with its K ranges split
// across blocks), whose bits are the fused kernel's (the runtime's permuted Mconv6 output order,
// pack_x3 with the Mconv7 channel map; x3_canonical_order over the waves).
bool x3_fused67_grid(const ConvLaunch& c) {
  const int bpx = c.cout == 512 ? 128 : c.cout == 256 ? 256 : 512;
  const long long blocks = (long long)c.n * ((c.H * c.W + tile_pixels(c, bpx, x3_segmax(bpx)) - 1) /
                                             tile_pixels(c, bpx, x3_segmax(bpx)));
  return 2 * blocks >= device_cus();
}

double conv_x3_fused67_mfma_flops(const ConvLaunch& c) {
  const int bpx = c.cout == 512 ? 128 : c.cout == 256 ? 256 : 512;
  const double px = std::ceil((double)c.H * c.W / tile_pixels(c, bpx, x3_segmax(bpx))) * bpx * c.n;
  const double k6 = ((c.cin_chunks + 1) / 2) * 16.0;
  return 3.0 * 2.0 * px * ((double)c.cout * k6 + 32.0 * ((c.cout7 + 31) / 32) * c.cout);
}


// conv_x3_wr for the launches whose K ranges would run across blocks (x3_ranges), by default
// those with at most 4 ranges; ISLPOSE_X3_WR=0: the split-K launches + x3_splitk_reduce (A/B),
// =2: also the small grids without K ranges (one wave per block summing the whole K; A/B), =3:
// every range count; ISLPOSE_X3_WR_WN=2: 64-pixel tiles (two 32-pixel accumulator tiles per wave
// sharing the weight fragments).  Read per launch.
static int x3_wr_mode() {
  const char* e = getenv("ISLPOSE_X3_WR");
  return e ? atoi(e) : 1;
}

template <int KS, int WN, int DEPTH>
static hipError_t launch_wr_t(const ConvLaunch& c, int S, hipStream_t s) {
  constexpr int P = KS / 2;
  if (c.in_pad < P) { set_error("conv_x3_wr: input ring narrower than kernel radius"); return hipErrorInvalidValue; }
  if ((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) { set_error("conv_x3_wr: slice not on a chunk"); return hipErrorInvalidValue; }
  if (!c.wx3 || !c.range_flag) { set_error("conv_x3_wr: split weights / range flag missing"); return hipErrorInvalidValue; }
  if (c.hpool || c.vin || c.fold || c.fold_out || c.cout7 > 0) {
    set_error("conv_x3_wr: plain layers only (no fused pool, fold or pair)");
    return hipErrorInvalidValue;
  }
  const int pairs = (c.cin_chunks + 1) / 2;
  if (S < 1 || S > 8 || S > pairs || c.bco % 32 || c.bco <= 0) { set_error("conv_x3_wr: bad range count / tile"); return hipErrorInvalidValue; }
  X3Args a{};
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.wpk = (const f16x8*)c.wx3; a.bias = c.bias; a.slope = c.slope;
  a.range_flag = c.range_flag;
  a.wscale_inv = c.wscale_inv;
  a.in_pad = c.in_pad; a.out_pad = c.out_pad;
  a.H = c.H; a.W = c.W; a.cin_chunks = c.cin_chunks; a.pairs = pairs; a.cout = c.cout;
  a.co_tiles = (c.cout + 31) / 32;
  a.tpx = 32 * WN;
  a.px_tiles = (c.H * c.W + a.tpx - 1) / a.tpx;
  a.act = c.act;
  a.ksplit = S;
  a.nfr = c.n;
  a.bco_pack = c.bco;
  a.dbg = c.dbg;   // development stamps (tools/convbench); never set by the runtime
  const long long nb = (long long)c.n * a.px_tiles * a.co_tiles;
  if (nb <= 0 || nb > 0x7fffffff) { set_error("conv_x3_wr: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
  t_last_variant = x3_variant_code(8 | (S > 1 ? 1024 : 0), KS, 32 * WN, 32);
  hipLaunchKernelGGL((conv_x3_wr<KS, WN, DEPTH>), dim3(a.nblocks), dim3(64 * S), 0, s, a);
  return hipGetLastError();
}

static hipError_t launch_x3_wr(const ConvLaunch& c, int S, hipStream_t s) {
  const char* e = getenv("ISLPOSE_X3_WR_WN");
  const bool wn2 = e && e[0] == '2';
  switch (c.ks) {
    case 1: return wn2 ? launch_wr_t<1, 2, 8>(c, S, s) : launch_wr_t<1, 1, 12>(c, S, s);
    case 3: return wn2 ? launch_wr_t<3, 2, 8>(c, S, s) : launch_wr_t<3, 1, 12>(c, S, s);
    case 7: return wn2 ? launch_wr_t<7, 2, 8>(c, S, s) : launch_wr_t<7, 1, 12>(c, S, s);
  }
  set_error("conv_x3_wr: unsupported kernel size");
  return hipErrorInvalidValue;
}

hipError_t launch_conv_x3(const ConvLaunch& c0, hipStream_t s) {
  if (c0.cout7 > 0) return launch_x3_fused67(c0, s);
  ConvLaunch c = c0;
  const X3Ranges r = x3_ranges(c);
  c.ksplit = r.S;
  // wave ranges where a 1x1 / 3x3 layer has at most 4 K ranges: with 8 a block's 8 waves load 2x
  // the operand bytes per CU of the split-K blocks (no sharing between ranges), and in the net the
  // c384 / c288 stage layers ran 20-35 % slower on it (profiles/r05/r5c/ops_*.txt); a 7x7 range
  // is 98 taps long for one wave (the hand's 184-pixel scale: C3 109.4 -> 107.5 frames/s on it,
  // profiles/r05/r5n/)
  if (r.across_blocks && !c.fold_out && (x3_wr_mode() >= 3 || (x3_wr_mode() >= 1 && r.S <= 4 && c.ks <= 3)))
    return launch_x3_wr(c, r.S, s);
  if (x3_wr_mode() == 2 && r.S == 1 && c.ks <= 3 && !c.hpool && !c.vin && !c.fold && !x3_big_tiles(c) &&
      x3_7x7_bpx(c) == 128)
    return launch_x3_wr(c, 1, s);
  if (r.across_blocks) {
    if (!c.ws || (size_t)r.S * c.n * ((c.cout + 7) / 8) * 8 * c.H * c.W > c.ws_floats) {
      set_error("conv_x3: split-K workspace too small");
      return hipErrorInvalidValue;
    }
  } else {
    c.ws = nullptr;        // in-block ranges (or none)
  }
  switch (c.ks) {
    case 1: return launch_ks<1>(c, s);
    case 3: return launch_ks<3>(c, s);
    case 7: return launch_ks<7>(c, s);
  }
  set_error("conv_x3: unsupported kernel size");
  return hipErrorInvalidValue;
}

}  // namespace isl
