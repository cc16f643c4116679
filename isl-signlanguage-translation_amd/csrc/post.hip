// Post-network kernels of Body.__call__ (src/body.py:64-235) and
// Hand.__call__ (src/hand.py:51-74):
//
//   resize_sep_kernel  cv2.resize INTER_CUBIC of the low-res maps (x8, crop,
//                      to frame size), fp32, OpenCV operation order; planar
//                      tiles, horizontal pass per source row staged in LDS
//   blur_nms_kernel    gaussian_filter(sigma=3) in fp64 (scipy order) fused
//                      with the 4-neighbour NMS -> one 64-bit mask word per
//                      (row, 64 columns), written by a wave ballot
//   compact_kernel     raster-order peak lists (np.nonzero order) + scores
//   limb_kernel        PAF line integral for every (A,B) pair of one limb
//                      (PAF sampled on demand from the low-res / intermediate
//                      maps), stable score sort, greedy matching -- one
//                      workgroup per (limb, frame)
//   assemble_kernel    person assembly, merge / delete, pruning (body.py:164-
//                      232) -- one lane per frame
//
// Every floating-point expression follows the reference's evaluation order;
// the file is built with -ffp-contract=off so no FMA is formed.
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <string>
#include <vector>

#include "internal.h"
#include "islpose.h"

namespace isl {

// scipy _gaussian_kernel1d(3, 0, 12), taps 0..12 (symmetric), from numpy
__constant__ double kGauss[13] = {
    0x1.105a329f98197p-3, 0x1.01a25f86eb137p-3, 0x1.b42a57d56c0bep-4, 0x1.4a614d1afd337p-4,
    0x1.bfde9c12bec92p-5, 0x1.0fa58939b528fp-5, 0x1.26defcaeb0202p-6, 0x1.1e6bccad344bap-7,
    0x1.f1e9915139406p-9, 0x1.8345966f69518p-10, 0x1.0d8a5ad43c165p-11, 0x1.4fbe39149e277p-13,
    0x1.763a210dfb306p-15};

// limb tables, body.py:111-126
__constant__ int kLimbs25[24][2] = {{1, 0}, {1, 2}, {2, 3}, {3, 4}, {1, 5}, {5, 6}, {6, 7}, {1, 8},
                                    {8, 9}, {9, 10}, {10, 11}, {8, 12}, {12, 13}, {13, 14}, {0, 15}, {0, 16},
                                    {15, 17}, {16, 18}, {11, 24}, {11, 22}, {14, 21}, {14, 19}, {22, 23}, {19, 20}};
__constant__ int kMap25[24][2] = {{30, 31}, {14, 15}, {16, 17}, {18, 19}, {22, 23}, {24, 25}, {26, 27}, {0, 1},
                                  {6, 7}, {2, 3}, {4, 5}, {8, 9}, {10, 11}, {12, 13}, {32, 33}, {34, 35},
                                  {36, 37}, {38, 39}, {50, 51}, {46, 47}, {44, 45}, {40, 41}, {48, 49}, {42, 43}};
__constant__ int kLimbsCoco[19][2] = {{1, 2}, {1, 5}, {2, 3}, {3, 4}, {5, 6}, {6, 7}, {1, 8}, {8, 9}, {9, 10}, {1, 11},
                                      {11, 12}, {12, 13}, {1, 0}, {0, 14}, {14, 16}, {0, 15}, {15, 17}, {2, 16}, {5, 17}};
__constant__ int kMapCoco[19][2] = {{12, 13}, {20, 21}, {14, 15}, {16, 17}, {22, 23}, {24, 25}, {0, 1},
                                    {2, 3},   {4, 5},   {6, 7},   {8, 9},   {10, 11}, {28, 29}, {30, 31},
                                    {34, 35}, {32, 33}, {36, 37}, {18, 19}, {26, 27}};

// ---------------------------------------------------------------------------
// cubic resize (OpenCV generic path; see oracle/cv_resize.py for the contract)
// ---------------------------------------------------------------------------



// channel c of map m (planar maps: cshift = 30, so chan(c) = c * cstr)
__device__ __forceinline__ long long chan_off(const MapSrc& m, int c) {
  return (long long)(c >> m.cshift) * m.cbig + (long long)(c & ((1 << m.cshift) - 1)) * m.cstr;
}

__device__ __forceinline__ void cubic_coeffs_f(float t, float c[4]) {
  const float A = -0.75f;
  const float tp1 = t + 1.f;
  c[0] = ((A * tp1 - 5.f * A) * tp1 + 8.f * A) * tp1 - 4.f * A;
  c[1] = ((A + 2.f) * t - (A + 3.f)) * t * t + 1.f;
  const float u = 1.f - t;
  c[2] = ((A + 2.f) * u - (A + 3.f)) * u * u + 1.f;
  c[3] = 1.f - c[0] - c[1] - c[2];
}

__device__ __forceinline__ void taps(int d, double scale, int n, int idx[4], float c[4]) {
  float f = (float)((d + 0.5) * scale - 0.5);
  const int s = (int)floorf(f);
  f -= (float)s;
  cubic_coeffs_f(f, c);
#pragma unroll
  for (int k = 0; k < 4; ++k) idx[k] = min(max(s + k - 1, 0), n - 1);
}

// one output element of resize `m`, with the row taps (yi, be) precomputed
__device__ __forceinline__ float sample_row(const MapSrc& m, int f, int c, const int yi[4], const float be[4], int x) {
  const float* b = m.base + f * m.fs + chan_off(m, c);
  int xi[4];
  float a[4];
  taps(x, m.scx, m.sw, xi, a);
  float hz[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float* r = b + yi[k] * m.ys;
    hz[k] = ((r[xi[0] * m.xs] * a[0] + r[xi[1] * m.xs] * a[1]) + r[xi[2] * m.xs] * a[2]) + r[xi[3] * m.xs] * a[3];
  }
  const int rowlen = m.dw * m.cn;
  if (x * m.cn + c < rowlen - rowlen % 4)
    return hz[0] * be[0] + (hz[1] * be[1] + (hz[2] * be[2] + hz[3] * be[3]));
  return ((hz[0] * be[0] + hz[1] * be[1]) + hz[2] * be[2]) + hz[3] * be[3];
}

__device__ __forceinline__ float sample(const MapSrc& m, int f, int c, int y, int x) {
  const float* b = m.base + f * m.fs + chan_off(m, c);
  if (m.identity) return b[y * m.ys + x * m.xs];
  int xi[4], yi[4];
  float a[4], be[4];
  taps(x, m.scx, m.sw, xi, a);
  taps(y, m.scy, m.sh, yi, be);
  float hz[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float* r = b + yi[k] * m.ys;
    hz[k] = ((r[xi[0] * m.xs] * a[0] + r[xi[1] * m.xs] * a[1]) + r[xi[2] * m.xs] * a[2]) + r[xi[3] * m.xs] * a[3];
  }
  const int rowlen = m.dw * m.cn;
  if (x * m.cn + c < rowlen - rowlen % 4)   // VResizeCubicVec_32f body (mul + add, SSE baseline)
    return hz[0] * be[0] + (hz[1] * be[1] + (hz[2] * be[2] + hz[3] * be[3]));
  return ((hz[0] * be[0] + hz[1] * be[1]) + hz[2] * be[2]) + hz[3] * be[3];   // scalar tail
}

// Separable tiled resize, planar output [n][nch][oh][ow] (f32, or f64 accumulation):
// a block covers RS_TY output rows x RS_TX output columns of one plane.  The
// horizontal pass is computed once per source row the tile needs (OpenCV's
// HResizeCubic, stored in LDS), then every output combines 4 of those rows
// (VResizeCubic) -- the same values OpenCV computes, with 4-5x fewer loads.
constexpr int RS_TY = 64, RS_TX = 256, RS_MAXR = 40;   // 64 rows: amortise the horizontal pass
// The vertical taps of the tile's output rows are computed once per block into LDS (they
// depend on the row only; per thread they were most of the vertical pass's VALU work), and
// the block is TX = 128 or 256 columns wide, whichever wastes fewer idle lanes on the
// output width (launch_resize): the same values, bit for bit.
// VU: vertical outputs per unrolled step; HU: source rows' loads in flight.  The arithmetic is
// the same either way.
// BM (mode 1, 64-row tiles of 128 columns): also the max |value| of every 16-row band x
// 64-column word of the output plane into bandmax[plane][oh / 16][ow / 64] (the blur's tile
// liveness, blur_tile: a tile whose window's bands stay below the threshold loads nothing)
// V4 (mode 1, TX = 128, not identity, ow % 4 == 0): the vertical pass by 4 adjacent columns x
// ty/4 rows per thread -- ds_read_b128 of the 4 LDS rows, one 16-byte store per output row (the
// HBM write path wants 16 bytes per lane) -- and with BM one band per thread (ty = 64).
constexpr int BM_ROWS = 16;
template <int TX, int VU = 1, int HU = 8, bool BM = false, bool V4 = false>
__global__ void __launch_bounds__(TX) resize_sep_kernel(MapSrc m, int nch, int oh, int ow, int ty_rows, int mode,
                                                         float inv_div_f, void* out, float* bandmax = nullptr,
                                                         const unsigned char* __restrict__ need = nullptr) {
  __shared__ float s_h[RS_MAXR][TX];
  __shared__ int4 s_yi[RS_TY];
  __shared__ float4 s_be[RS_TY];
  const int plane = blockIdx.x, f = plane / nch, c = plane - f * nch;
  // need (stage2_need_kernel): tiles no live blur window reads are not computed (their band
  // maxima are never read either: band_live_kernel requires the tile's live_mid first)
  if (need && !need[((size_t)plane * gridDim.y + blockIdx.y) * gridDim.z + blockIdx.z]) return;
  const int y0 = blockIdx.y * ty_rows, x = blockIdx.z * TX + threadIdx.x;
  const int ny = min(ty_rows, oh - y0);
  const float* b = m.base + (size_t)f * m.fs + chan_off(m, c);
  // source rows the tile needs: [r_lo, r_lo + nr)
  int r_lo = y0, nr = ny;
  if (!m.identity) {
    int lo[4], hi[4];
    float dummy[4];
    taps(y0, m.scy, m.sh, lo, dummy);
    taps(y0 + ny - 1, m.scy, m.sh, hi, dummy);
    r_lo = lo[0];
    nr = hi[3] - r_lo + 1;
    if ((int)threadIdx.x < ny) {
      int yi[4];
      float be[4];
      taps(y0 + threadIdx.x, m.scy, m.sh, yi, be);
      s_yi[threadIdx.x] = make_int4(yi[0] - r_lo, yi[1] - r_lo, yi[2] - r_lo, yi[3] - r_lo);
      s_be[threadIdx.x] = make_float4(be[0], be[1], be[2], be[3]);
    }
  }
  if (nr > RS_MAXR) __builtin_trap();   // the host sizes ty_rows so that this cannot happen
  if (x < ow) {
    if (m.identity) {
      for (int r = 0; r < nr; ++r) s_h[r][threadIdx.x] = b[(size_t)(r_lo + r) * m.ys + (size_t)x * m.xs];
    } else {
      int xi[4];
      float a[4];
      taps(x, m.scx, m.sw, xi, a);
      const long long o0 = xi[0] * m.xs, o1 = xi[1] * m.xs, o2 = xi[2] * m.xs, o3 = xi[3] * m.xs;
      // 8 rows' loads in flight at a time: the row loop is otherwise one L2 round trip per row
      // (Mode R post 1.60 -> 1.48 ms against a rolled loop, profiles/r03/resize_ab/)
#pragma unroll HU
      for (int r = 0; r < nr; ++r) {
        const float* row = b + (size_t)(r_lo + r) * m.ys;
        s_h[r][threadIdx.x] = ((row[o0] * a[0] + row[o1] * a[1]) + row[o2] * a[2]) + row[o3] * a[3];
      }
    }
  }
  __syncthreads();
  if constexpr (V4) {
    static_assert(TX == 128, "V4: 32 column groups x 4 row groups");
    const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const int xl = cg * 4, xv = blockIdx.z * TX + xl;
    const int rows = ty_rows / 4, t0 = rg * rows, t1 = min(t0 + rows, ny);
    const int rowlen = m.dw * m.cn, body = rowlen - rowlen % 4;
    bool sv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sv[j] = (xv + j) * m.cn + c < body;
    float bmx = 0.f;
#pragma unroll 2
    for (int t = t0; t < t1; ++t) {
      const int4 yi = s_yi[t];
      const float4 be = s_be[t];
      const float4 h0 = *reinterpret_cast<const float4*>(&s_h[yi.x][xl]);
      const float4 h1 = *reinterpret_cast<const float4*>(&s_h[yi.y][xl]);
      const float4 h2 = *reinterpret_cast<const float4*>(&s_h[yi.z][xl]);
      const float4 h3 = *reinterpret_cast<const float4*>(&s_h[yi.w][xl]);
      auto vc = [&](bool simd, float a0, float a1, float a2, float a3) {
        return simd ? a0 * be.x + (a1 * be.y + (a2 * be.z + a3 * be.w))   // VResizeCubicVec_32f body
                    : ((a0 * be.x + a1 * be.y) + a2 * be.z) + a3 * be.w;   // scalar tail
      };
      float4 v;
      v.x = vc(sv[0], h0.x, h1.x, h2.x, h3.x);
      v.y = vc(sv[1], h0.y, h1.y, h2.y, h3.y);
      v.z = vc(sv[2], h0.z, h1.z, h2.z, h3.z);
      v.w = vc(sv[3], h0.w, h1.w, h2.w, h3.w);
      if (xv < ow) {
        *reinterpret_cast<float4*>(&((float*)out)[((size_t)plane * oh + y0 + t) * ow + xv]) = v;
        if constexpr (BM) bmx = fmaxf(bmx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    }
    if constexpr (BM) {
      // this thread's rows are one band (ty = 64, y0 % 16 == 0): max over the word's 16 lanes
      for (int o = 8; o > 0; o >>= 1) bmx = fmaxf(bmx, __shfl_xor(bmx, o));
      const int words = (ow + 63) / 64, bands = (oh + BM_ROWS - 1) / BM_ROWS;
      if ((cg & 15) == 0 && xv < ow && t0 < ny)
        bandmax[((size_t)plane * bands + (y0 + t0) / BM_ROWS) * words + xv / 64] = bmx;
    }
    return;
  }
  if (!BM && x >= ow) return;   // (BM: every lane takes part in the band maxima's shuffles)
  const int rowlen = m.dw * m.cn, body = rowlen - rowlen % 4;
  const bool simd = x * m.cn + c < body;
  float bmx = 0.f;
#pragma unroll VU
  for (int t = 0; t < ny; ++t) {
    const int y = y0 + t;
    float v = 0.f;
    if (!BM || x < ow) {
      if (m.identity) {
        v = s_h[t][threadIdx.x];
      } else {
        const int4 yi = s_yi[t];
        const float4 be = s_be[t];
        const float h0 = s_h[yi.x][threadIdx.x], h1 = s_h[yi.y][threadIdx.x];
        const float h2 = s_h[yi.z][threadIdx.x], h3 = s_h[yi.w][threadIdx.x];
        v = simd ? h0 * be.x + (h1 * be.y + (h2 * be.z + h3 * be.w))   // VResizeCubicVec_32f body
                 : ((h0 * be.x + h1 * be.y) + h2 * be.z) + h3 * be.w;   // scalar tail
      }
      const size_t i = ((size_t)plane * oh + y) * ow + x;
      if (BM || mode == 1) {
        ((float*)out)[i] = v;
      } else {
        // mode | 8: the first scale -- the accumulator is the reference's np.zeros, so it
        // starts from +0.0 here instead of a memset pass (same bits, 0.0 + x included)
        double* o = (double*)out + i;
        const double o0 = (mode & 8) ? 0.0 : *o;
        const float q = v / inv_div_f;   // heatmap / len(multiplier), float32
        if ((mode & 7) == 2) *o = o0 + (o0 + (double)q);   // body.py:80, the doubling quirk
        else *o = o0 + (double)q;                          // hand.py:56
      }
    }
    if constexpr (BM) {
      bmx = fmaxf(bmx, fabsf(v));   // (0 past the plane's width)
      if (t % BM_ROWS == BM_ROWS - 1 || t == ny - 1) {   // a band ends (uniform): max over the wave's 64 columns
        float w = bmx;
        for (int o = 32; o > 0; o >>= 1) w = fmaxf(w, __shfl_xor(w, o));
        const int words = (ow + 63) / 64, bands = (oh + BM_ROWS - 1) / BM_ROWS;
        if ((threadIdx.x & 63) == 0 && blockIdx.z * TX + (threadIdx.x & ~63) < ow)
          bandmax[((size_t)plane * bands + y / BM_ROWS) * words + (blockIdx.z * TX + threadIdx.x) / 64] = w;
        bmx = 0.f;
      }
    }
  }
}

// The hand average over the scales in one pass (hand.py:51-56): for every output pixel
// the final resize of each scale (resize_sep_kernel's arithmetic: horizontal pass into
// LDS, vertical combine) and heatmap_avg += heatmap / len(multiplier) in scale order in
// fp64 registers, one store.  The same bits as a mode-(3|8) pass then ns-1 mode-3 passes,
// without their ns read-modify-write sweeps of the fp64 average.
constexpr int RA_TY = 16;   // output rows per block (fp64 accumulators in registers)
struct MapSrcN {   // up to MAX_SCALES (8) scales
  MapSrc m[8];
};
__global__ void __launch_bounds__(256) resize_acc_kernel(MapSrcN ms, int ns, int nch, int oh, int ow, int ty_rows,
                                                         float div_f, int quirk, double* out) {
  __shared__ float s_h[RS_MAXR][RS_TX];
  __shared__ int4 s_yi[RA_TY];          // vertical taps of the tile's rows, per scale (as resize_sep_kernel)
  __shared__ float4 s_be[RA_TY];
  const int plane = blockIdx.x, f = plane / nch, c = plane - f * nch;
  const int y0 = blockIdx.y * ty_rows, x = blockIdx.z * RS_TX + threadIdx.x;
  const int ny = min(ty_rows, oh - y0);
  double acc[RA_TY];
#pragma unroll
  for (int t = 0; t < RA_TY; ++t) acc[t] = 0.0;
  for (int si = 0; si < ns; ++si) {
    const MapSrc& m = ms.m[si];
    const float* b = m.base + (size_t)f * m.fs + chan_off(m, c);
    int r_lo = y0, nr = ny;
    if (!m.identity) {
      int lo[4], hi[4];
      float dummy[4];
      taps(y0, m.scy, m.sh, lo, dummy);
      taps(y0 + ny - 1, m.scy, m.sh, hi, dummy);
      r_lo = lo[0];
      nr = hi[3] - r_lo + 1;
    }
    if (nr > RS_MAXR) __builtin_trap();   // the host sizes ty_rows so that this cannot happen
    __syncthreads();                      // the previous scale's vertical pass is done with s_h
    if (!m.identity && (int)threadIdx.x < ny) {
      int yi[4];
      float be[4];
      taps(y0 + threadIdx.x, m.scy, m.sh, yi, be);
      s_yi[threadIdx.x] = make_int4(yi[0] - r_lo, yi[1] - r_lo, yi[2] - r_lo, yi[3] - r_lo);
      s_be[threadIdx.x] = make_float4(be[0], be[1], be[2], be[3]);
    }
    if (x < ow) {
      if (m.identity) {
        for (int r = 0; r < nr; ++r) s_h[r][threadIdx.x] = b[(size_t)(r_lo + r) * m.ys + (size_t)x * m.xs];
      } else {
        int xi[4];
        float a[4];
        taps(x, m.scx, m.sw, xi, a);
        const long long o0 = xi[0] * m.xs, o1 = xi[1] * m.xs, o2 = xi[2] * m.xs, o3 = xi[3] * m.xs;
#pragma unroll 8
        for (int r = 0; r < nr; ++r) {
          const float* row = b + (size_t)(r_lo + r) * m.ys;
          s_h[r][threadIdx.x] = ((row[o0] * a[0] + row[o1] * a[1]) + row[o2] * a[2]) + row[o3] * a[3];
        }
      }
    }
    __syncthreads();
    if (x < ow) {
      const int rowlen = m.dw * m.cn, body = rowlen - rowlen % 4;
      const bool simd = x * m.cn + c < body;
#pragma unroll
      for (int t = 0; t < RA_TY; ++t) {
        if (t >= ny) break;
        float v;
        if (m.identity) {
          v = s_h[t][threadIdx.x];
        } else {
          const int4 yi = s_yi[t];
          const float4 be = s_be[t];
          const float h0 = s_h[yi.x][threadIdx.x], h1 = s_h[yi.y][threadIdx.x];
          const float h2 = s_h[yi.z][threadIdx.x], h3 = s_h[yi.w][threadIdx.x];
          v = simd ? h0 * be.x + (h1 * be.y + (h2 * be.z + h3 * be.w))
                   : ((h0 * be.x + h1 * be.y) + h2 * be.z) + h3 * be.w;
        }
        const float q = v / div_f;      // heatmap / len(multiplier), float32
        // from np.zeros (0.0 + x included): hand.py:56, or body.py:80's doubling quirk
        acc[t] = quirk ? acc[t] + (acc[t] + (double)q) : acc[t] + (double)q;
      }
    }
  }
  if (x >= ow) return;
#pragma unroll
  for (int t = 0; t < RA_TY; ++t) {
    if (t >= ny) break;
    out[((size_t)plane * oh + y0 + t) * ow + x] = acc[t];
  }
}

// ---------------------------------------------------------------------------
// fp64 blur + NMS
// ---------------------------------------------------------------------------

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // scipy 'reflect' (d c b a | a b c d | d c b a), periodic for short lines
  const int p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - 1 - i;
}

// Tile: 16 output rows x 192 output columns (3 mask words).  The NMS needs g on
// a one-pixel ring, the blur a 12-pixel apron:
//   axis 0: one thread per column (218 = 192+2+24), the 42 input rows of that
//           column held in registers -> 18 rows of v into LDS
//   axis 1: one thread per 14-column run of one of the 18 rows, 38 v values in
//           registers -> g into LDS
//   NMS:    one wave per (row, 64-column word), ballot -> mask word.
constexpr int NMS_TY = 16, NMS_TX = 192, NMS_R = 12;
constexpr int NMS_VR = NMS_TY + 2;                 // g / v rows (1-px ring)
constexpr int NMS_VC = NMS_TX + 2 + 2 * NMS_R;     // v columns (218)
constexpr int NMS_GC = NMS_TX + 2;                 // g columns (194)
constexpr int NMS_IR = NMS_VR + 2 * NMS_R;         // input rows (42)
constexpr int NMS_SEG = 14;                        // g outputs per thread in the horizontal pass

// Fused single-scale source (FUSED = true): the planes are not materialised; the
// tile's input window is resized on the fly from the low-resolution map `m`
// (stage-1 cv2.resize x8, cropped: body.py:68-73 when the net input is the frame),
// with resize_sep_kernel's exact operation order.  Only scale 1/8 is fused.
constexpr int NMS_SRC_ROWS = 16;
constexpr int NMS_SRC_COLS = 48;                   // source columns (218 / 8 + 5 = 33 at scale 1/8; 42 at 1/5.9)
// The wide window (Mode R at 368 x 656: the stage-2 resize is x2, a tile reads ~26 x 114 source
// values): 72 KB of LDS per block, two blocks per CU, against writing and re-reading 0.8 GB of
// full-resolution heat planes per 32 frames -- measured slower, opt-in (fused_wide_enabled).
constexpr int NMS_WSRC_ROWS = 28;
constexpr int NMS_WSRC_COLS = 120;

// [min, max] of reflect_idx(i, n) over i in [lo, hi]
__device__ __forceinline__ void reflect_range(int lo, int hi, int n, int* a, int* b) {
  if (hi - lo + 1 >= n) { *a = 0; *b = n - 1; return; }          // may wrap: take the whole line
  if (lo < 0) { *a = 0; *b = max(hi, -lo - 1); return; }           // (one edge only: the window is < n)
  if (hi >= n) { *a = min(lo, 2 * n - 1 - hi); *b = n - 1; return; }
  *a = lo; *b = hi;
}

// low-res window [sr0, sr0+nsr) x [sc0, sc0+nsc) that the fused tile at (y0, x0) reads
__device__ __forceinline__ void fused_window(const MapSrc& m, int H, int W, int y0, int x0, int* sr0, int* nsr,
                                             int* sc0, int* nsc) {
  // the window's rows / columns are reflect(y0-13 .. y0+28) / reflect(x0-13 .. x0+204);
  // cubic taps are monotone in the index, so [taps(min)[0], taps(max)[3]] covers them
  int rlo, rhi, clo, chi;
  reflect_range(y0 - 1 - NMS_R, y0 - 2 - NMS_R + NMS_IR, H, &rlo, &rhi);
  reflect_range(x0 - 1 - NMS_R, x0 - 2 - NMS_R + NMS_VC, W, &clo, &chi);
  int t0[4], t1[4], u0[4], u1[4];
  float dmy[4];
  taps(rlo, m.scy, m.sh, t0, dmy);
  taps(rhi, m.scy, m.sh, t1, dmy);
  taps(clo, m.scx, m.sw, u0, dmy);
  taps(chi, m.scx, m.sw, u1, dmy);
  *sr0 = t0[0];
  *nsr = t1[3] - t0[0] + 1;
  *sc0 = u0[0];
  *nsc = u1[3] - u0[0] + 1;
}
// Early out, exact: |resized| <= max|low| * (sum|cubic taps|)^2, and fp32 rounding is
// covered by the 1.9 / 1.890625 margin; then |g| <= max|resized| * (1 + 1e-13).
constexpr double CUBIC_ABS_SUM_SQ = 1.890625;      // max over t of (sum_k |cubic_k(t)|)^2, A = -0.75

// The fp32 filter (default): the two passes in packed fp32 with fused multiply-adds
// (v_pk_fma_f32: two outputs per instruction, 25 instructions per output pair against 37
// fp64 per output), a column pair per thread in the vertical pass, a row pair per thread in
// the horizontal one.  Bound: each tap of the scipy recurrence goes through at most 14
// roundings (weight, pair sum, 12 accumulations) and the weights are positive with sum 1,
// so with M = max |in| over the tile's window |v32 - v| <= 14.01 u M and |g32 - g| <= 28.1 u M
// (u = 2^-24; the fp64 passes and the fp32 rounding of fp64 planes add < 1.1 u M).  With
// eps = 2^-18 M (64 u M) a pixel whose every comparison clears the margin (g vs thre by eps,
// g vs a neighbour by 2 eps; compared in fp32 with the margin doubled, see the NMS below) has
// the fp64 decision; a tile with any pixel inside a margin
// (a peak at the threshold, two near-equal neighbours at a peak: rare) is appended to a list
// that a second launch re-runs on the exact fp64 passes (blur_tile_exact), which rewrite all
// of the tile's words.  The mask bits are the fp64 ones either way.  The filter's tile keeps
// no fp64 planes and no staged window: 19 KB of LDS (37 KB fused) against 33 / 52 KB.
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr double kGaussC[13] = {
    0x1.105a329f98197p-3, 0x1.01a25f86eb137p-3, 0x1.b42a57d56c0bep-4, 0x1.4a614d1afd337p-4,
    0x1.bfde9c12bec92p-5, 0x1.0fa58939b528fp-5, 0x1.26defcaeb0202p-6, 0x1.1e6bccad344bap-7,
    0x1.f1e9915139406p-9, 0x1.8345966f69518p-10, 0x1.0d8a5ad43c165p-11, 0x1.4fbe39149e277p-13,
    0x1.763a210dfb306p-15};
constexpr float kGaussF[13] = {(float)kGaussC[0],  (float)kGaussC[1],  (float)kGaussC[2],  (float)kGaussC[3],
                               (float)kGaussC[4],  (float)kGaussC[5],  (float)kGaussC[6],  (float)kGaussC[7],
                               (float)kGaussC[8],  (float)kGaussC[9],  (float)kGaussC[10], (float)kGaussC[11],
                               (float)kGaussC[12]};
constexpr double BLUR_EPS_REL = 0x1p-18;
constexpr int NMS_CP = NMS_VC / 2;                  // column pairs of the filter's vertical pass (109)
constexpr int NMS_VH = NMS_VR / 2;                  // v rows per thread (two waves' worth per half)
constexpr int NMS_HSEG = 7, NMS_HRUNS = 28;         // filter horizontal pass: 9 row pairs x 28 runs of 7
static_assert(NMS_VC % 2 == 0 && NMS_VR % 2 == 0 && NMS_CP <= 128 && NMS_HSEG * NMS_HRUNS >= NMS_GC &&
                  NMS_VR / 2 * NMS_HRUNS <= 256,
              "filter tiling");

// Development build only: per-tile phase stamps of the blur (tools/tile_prof.py) -- 10 u64
// per tile: wall clock at start / end, shader clock at start, after the prologue (band or
// low-res bound, the fused horizontal resize), after the window, after the vertical pass,
// after the horizontal pass, after the NMS, the fallback flag (the filter appended the
// tile), at the exact re-run's end (0 where a phase never ran)
#ifdef ISLPOSE_DEV
__device__ unsigned long long* g_tile_prof = nullptr;
#define TPROF(k, v)                                                                               \
  do {                                                                                            \
    if (g_tile_prof && tid == 0) {                                                                \
      const long long tix =                                                                       \
          ((long long)plane * ((H + NMS_TY - 1) / NMS_TY) + by) * ((W + NMS_TX - 1) / NMS_TX) + bx; \
      g_tile_prof[tix * 10 + (k)] = (v);                                                          \
    }                                                                                             \
  } while (0)
__device__ unsigned long long* g_asm_prof = nullptr;   // assemble_kernel phases: 8 u64 per frame
#define ASTAMP(k)                                                       \
  do {                                                                  \
    if (g_asm_prof && lane == 0) g_asm_prof[(size_t)f * 8 + (k)] = clock64(); \
  } while (0)
#else
#define TPROF(k, v) \
  do {              \
  } while (0)
#define ASTAMP(k) \
  do {            \
  } while (0)
#endif

// The band-maxima early out shared by both tile functions (bandmax: resize_sep_kernel's max
// |value| per 16-row band x 64-column word): the window's rows and columns, reflected, lie in
// those bands and words, so the exact blur bound below holds with their maximum.  Wave 0
// decides; true = the tile is dead.
__device__ __forceinline__ bool band_dead(const float* __restrict__ bandmax, int plane, int H, int W, int words, int y0,
                                          int x0, double thre, int* s_flag) {
  const int tid = threadIdx.x;
  if (tid == 0) *s_flag = 0;
  __syncthreads();
  if (tid < 64) {
    int rlo, rhi, clo, chi;
    reflect_range(y0 - 1 - NMS_R, y0 - 2 - NMS_R + NMS_IR, H, &rlo, &rhi);
    reflect_range(x0 - 1 - NMS_R, x0 - 2 - NMS_R + NMS_VC, W, &clo, &chi);
    const int b0 = rlo / BM_ROWS, nb = rhi / BM_ROWS - b0 + 1, w0 = clo / 64, nw = chi / 64 - w0 + 1;
    const int bands = (H + BM_ROWS - 1) / BM_ROWS;
    const bool all = nb * nw > 64;             // (tiny planes: no early out)
    float v = 0.f;
    if (tid < nb * nw) v = bandmax[((size_t)plane * bands + b0 + tid / nw) * words + w0 + tid % nw];
    float mx = all ? 1e30f : v;
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (tid == 0 && (double)mx >= thre * (1.0 - 1e-9)) *s_flag = 1;
  }
  __syncthreads();
  const bool dead = !*s_flag;
  __syncthreads();   // everyone has read the flag before it is reused
  return dead;
}

// The fused single-scale prologue: the low-res window into LDS, the exact low-res bound
// (false: the tile is dead), then the horizontal cubic pass of every window column and the
// vertical taps of the window's rows (resize_sep_kernel's order).
template <int WR, int WC>
__device__ __forceinline__ bool fused_prologue(const MapSrc& m, int nch, int plane, int H, int W, int y0, int x0,
                                               double thre, float (*s_low)[WC], float (*s_hz)[NMS_VC], int4* s_ti,
                                               float4* s_tb, int* s_flag) {
  const int tid = threadIdx.x;
  const int f = plane / nch, c = plane - f * nch;
  const float* b = m.base + (size_t)f * m.fs + chan_off(m, c);
  int sr0, nsr, sc0, nsc;
  fused_window(m, H, W, y0, x0, &sr0, &nsr, &sc0, &nsc);
  if (nsr > WR) __builtin_trap();   // the host picks a window that holds the tile's source rows
  // the low-res window is staged in LDS: one coalesced pass, reused by the resize
  if (nsc > WC) __builtin_trap();
  if (tid == 0) *s_flag = 0;
  __syncthreads();
  float amax = 0.f;
  for (int i = tid; i < nsr * nsc; i += 256) {
    const int r = i / nsc, cc = i - r * nsc;
    const float v = b[(size_t)(sr0 + r) * m.ys + (size_t)(sc0 + cc) * m.xs];
    s_low[r][cc] = v;
    amax = fmaxf(amax, fabsf(v));
  }
  if ((double)amax * 1.9 >= thre * (1.0 - 1e-9)) *s_flag = 1;
  __syncthreads();
  const bool live_lr = *s_flag != 0;
  __syncthreads();   // everyone has read the flag before it is reused
  if (!live_lr) return false;
  if (tid < NMS_VC) {
    // horizontal cubic pass for the window column (OpenCV HResizeCubic order)
    const int xx = reflect_idx(x0 - 1 - NMS_R + tid, W);
    int xi[4];
    float a[4];
    taps(xx, m.scx, m.sw, xi, a);
    const int i0 = xi[0] - sc0, i1 = xi[1] - sc0, i2 = xi[2] - sc0, i3 = xi[3] - sc0;
    for (int r = 0; r < nsr; ++r) {
      const float* row = s_low[r];
      s_hz[r][tid] = ((row[i0] * a[0] + row[i1] * a[1]) + row[i2] * a[2]) + row[i3] * a[3];
    }
  } else {
    // vertical taps of the window's 42 rows, once per block (the 38 idle lanes)
    for (int r = tid - NMS_VC; r < NMS_IR; r += 256 - NMS_VC) {
      int yi[4];
      float be[4];
      taps(reflect_idx(y0 - 1 - NMS_R + r, H), m.scy, m.sh, yi, be);
      s_ti[r] = make_int4(yi[0] - sr0, yi[1] - sr0, yi[2] - sr0, yi[3] - sr0);
      s_tb[r] = make_float4(be[0], be[1], be[2], be[3]);
    }
  }
  __syncthreads();
  return true;
}

// window value of the fused path: resize_sep_kernel's vertical combine (VResizeCubicVec_32f
// body / scalar tail) of window row r, column t (plane column xx)
__device__ __forceinline__ float fused_value(const MapSrc& m, int c, float (*s_hz)[NMS_VC], const int4* s_ti,
                                             const float4* s_tb, int r, int t, int xx) {
  const int4 yi = s_ti[r];
  const float4 be = s_tb[r];
  const float h0 = s_hz[yi.x][t], h1 = s_hz[yi.y][t], h2 = s_hz[yi.z][t], h3 = s_hz[yi.w][t];
  const int rowlen = m.dw * m.cn;
  return xx * m.cn + c < rowlen - rowlen % 4 ? h0 * be.x + (h1 * be.y + (h2 * be.z + h3 * be.w))
                                             : ((h0 * be.x + h1 * be.y) + h2 * be.z) + h3 * be.w;
}

// the exact fp64 passes (scipy's order) of one tile
// planes: [n*nparts][H][W] (T = float or double); mask: [n*nparts][H][words]
template <typename T, bool FUSED, int WR = NMS_SRC_ROWS, int WC = NMS_SRC_COLS>
__device__ __forceinline__ void blur_tile_exact(const T* __restrict__ planes, int H, int W, int words,
                                                unsigned long long* __restrict__ mask, double thre, int mode_hand,
                                                const MapSrc& m, int nch, int plane, int by, int bx,
                                                const float* __restrict__ bandmax) {
  // one LDS tile: v (axis-0 result), then g written in place over it (the
  // horizontal pass holds its v run in registers across a barrier) -> 31 KB,
  // so 4 blocks fit a CU and hide each other's load latency
  __shared__ double s_v[NMS_VR][NMS_VC];
  __shared__ float s_hz[FUSED ? WR : 1][NMS_VC];
  __shared__ int4 s_ti[FUSED ? NMS_IR : 1];
  __shared__ float s_low[FUSED ? WR : 1][WC];
  __shared__ float4 s_tb[FUSED ? NMS_IR : 1];
  __shared__ int s_live;
  __shared__ double s_cmax[NMS_VC];   // max |in| of every window column (word liveness)
  __shared__ int s_wlive[3];
  double (*s_g)[NMS_VC] = s_v;
  const int y0 = by * NMS_TY, x0 = bx * NMS_TX;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  auto zero_masks = [&]() {
    for (int it = wave; it < NMS_TY * 3; it += 4) {
      const int y = y0 + it / 3, wi = bx * 3 + it % 3;
      if (lane == 0 && y < H && wi < words) mask[((size_t)plane * H + y) * words + wi] = 0ull;
    }
  };
  if constexpr (!FUSED) {
    if (bandmax && band_dead(bandmax, plane, H, W, words, y0, x0, thre, &s_live)) {
      zero_masks();
      return;
    }
  } else {
    if (!fused_prologue<WR, WC>(m, nch, plane, H, W, y0, x0, thre, s_low, s_hz, s_ti, s_tb, &s_live)) {
      zero_masks();
      return;
    }
  }
  if (tid == 0) s_live = 0;
  __syncthreads();
  // axis 0 (NI_Correlate1D, symmetric): o = c*w0; for j = 12..1: o += (a[-j] + a[+j]) * w[j]
  double in[NMS_IR];
  if (tid < NMS_VC) {
    const int xx = reflect_idx(x0 - 1 - NMS_R + tid, W);
    double amax = 0.0;
#pragma unroll
    for (int r = 0; r < NMS_IR; ++r) {
      if constexpr (!FUSED)
        in[r] = (double)planes[(size_t)plane * H * W + (size_t)reflect_idx(y0 - 1 - NMS_R + r, H) * W + xx];
      else
        in[r] = (double)fused_value(m, plane % nch, s_hz, s_ti, s_tb, r, tid, xx);
      amax = fmax(amax, fabs(in[r]));
    }
    s_cmax[tid] = amax;
    // Early out, exact: every g of the tile is a positive-weight average (weights sum
    // to 1) of these inputs, so |g| <= max|in| * (1 + 1e-13) in fp64.  When that stays
    // below the threshold no pixel can pass `g > thre` and the tile's mask is zero.
    if (amax >= thre * (1.0 - 1e-9)) s_live = 1;
  }
  __syncthreads();
  if (!s_live) {
    zero_masks();
    return;
  }
  // Word liveness, the same exact bound per 64-column mask word: word w's outputs (tile
  // columns 64w..64w+63) read g on columns 64w..64w+65 (NMS ring), i.e. window columns
  // 64w..64w+89 of every input row; when those stay below the threshold the word is
  // zero and neither its vertical nor its horizontal pass runs.
  if (tid < 3) {
    double mx = 0.0;
    for (int t = 64 * tid; t <= 64 * tid + 89 && t < NMS_VC; ++t) mx = fmax(mx, s_cmax[t]);
    s_wlive[tid] = mx >= thre * (1.0 - 1e-9);
  }
  __syncthreads();
  const bool wl0 = s_wlive[0], wl1 = s_wlive[1], wl2 = s_wlive[2];
  // window column t is needed by a live word
  auto col_needed = [&](int t) {
    return (wl0 && t <= 89) || (wl1 && t >= 64 && t <= 153) || (wl2 && t >= 128);
  };
  if (tid < NMS_VC && col_needed(tid)) {
#pragma unroll
    for (int r = 0; r < NMS_VR; ++r) {
      double o = in[r + NMS_R] * kGauss[0];
#pragma unroll
      for (int j = NMS_R; j >= 1; --j) o = o + (in[r + NMS_R - j] + in[r + NMS_R + j]) * kGauss[j];
      s_v[r][tid] = o;
    }
  }
  __syncthreads();
  // axis 1, same recurrence along the row
  {
    constexpr int SEGS = (NMS_GC + NMS_SEG - 1) / NMS_SEG;   // 14 runs per row, 252 threads
    const int r = tid / SEGS, c0 = (tid - r * SEGS) * NMS_SEG;
    // g columns c0..c0+13 overlap a live word's g range [64w, 64w+65]; the run's other
    // columns may read v never computed -- their g is never read
    const int c1 = c0 + NMS_SEG - 1;
    const bool act = tid < NMS_VR * SEGS &&
                     ((wl0 && c0 <= 65) || (wl1 && c1 >= 64 && c0 <= 129) || (wl2 && c1 >= 128));
    double v[NMS_SEG + 2 * NMS_R];
    if (act) {
#pragma unroll
      for (int k = 0; k < NMS_SEG + 2 * NMS_R; ++k) v[k] = c0 + k < NMS_VC ? s_v[r][c0 + k] : 0.0;
    }
    __syncthreads();   // every v run is in registers: g may overwrite the tile
    if (act) {
#pragma unroll
      for (int k = 0; k < NMS_SEG; ++k) {
        double o = v[k + NMS_R] * kGauss[0];
#pragma unroll
        for (int j = NMS_R; j >= 1; --j) o = o + (v[k + NMS_R - j] + v[k + NMS_R + j]) * kGauss[j];
        if (c0 + k < NMS_GC) s_g[r][c0 + k] = o;
      }
    }
  }
  __syncthreads();
  // one wave per (row, 64-column word) -> one 64-bit mask word
#pragma unroll 2
  for (int q = 0; q < NMS_TY * 3 / 4; ++q) {
    const int it = wave + 4 * q;
    const int ty = it / 3, wd = it - ty * 3;
    const int y = y0 + ty, cx = wd * 64 + lane, x = x0 + cx;
    bool pk = false;
    const double g = s_g[ty + 1][cx + 1];   // (the reads lie in the tile: unconditional)
    const double gu = s_g[ty][cx + 1], gd = s_g[ty + 2][cx + 1], gl = s_g[ty + 1][cx], gr = s_g[ty + 1][cx + 2];
    if (y < H && x < W && (wd == 0 ? wl0 : wd == 1 ? wl1 : wl2)) {
      if (mode_hand) {
        pk = g > thre;                                  // hand.py:62 binary map
      } else {
        const double up = y > 0 ? gu : 0.0;
        const double dn = y + 1 < H ? gd : 0.0;
        const double lf = x > 0 ? gl : 0.0;
        const double rt = x + 1 < W ? gr : 0.0;
        pk = g >= up && g >= dn && g >= lf && g >= rt && g > thre;   // body.py:99-100
      }
    }
    const unsigned long long word = __ballot(pk);
    const int wi = bx * 3 + wd;
    if (lane == 0 && y < H && wi < words) mask[((size_t)plane * H + y) * words + wi] = word;
  }
  TPROF(9, clock64());
}

// the fp32 filter of one tile; undecided tiles are appended to amb (see above)
template <typename T, bool FUSED, int WR = NMS_SRC_ROWS, int WC = NMS_SRC_COLS>
__device__ __forceinline__ void blur_tile_filter(const T* __restrict__ planes, int H, int W, int words,
                                                 unsigned long long* __restrict__ mask, double thre, int mode_hand,
                                                 const MapSrc& m, int nch, int plane, int by, int bx,
                                                 const float* __restrict__ bandmax, int* __restrict__ amb,
                                                 int* __restrict__ amb_count, int tile_id, int margin_mode) {
  // v, then g in place (15.7 KB); fused: over the low-res window, which only the prologue's
  // horizontal pass reads
  constexpr int U = NMS_VR * NMS_VC > (FUSED ? WR * WC : 1) ? NMS_VR * NMS_VC : WR * WC;
  __shared__ float s_u[U];
  float(*s_vf)[NMS_VC] = reinterpret_cast<float(*)[NMS_VC]>(s_u);
  float(*s_low)[WC] = reinterpret_cast<float(*)[WC]>(s_u);
  __shared__ float s_hz[FUSED ? WR : 1][NMS_VC];
  __shared__ int4 s_ti[FUSED ? NMS_IR : 1];
  __shared__ float4 s_tb[FUSED ? NMS_IR : 1];
  __shared__ double s_cmax[2][NMS_VC];          // max |in| of every window column, per row half
  __shared__ double s_M;                        // max |in| over the window (the margin)
  __shared__ int s_live, s_amb;
  __shared__ int s_wlive[3];
  const int y0 = by * NMS_TY, x0 = bx * NMS_TX;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  TPROF(0, wall_clock64());
  TPROF(2, clock64());
  auto zero_masks = [&]() {
    for (int it = wave; it < NMS_TY * 3; it += 4) {
      const int y = y0 + it / 3, wi = bx * 3 + it % 3;
      if (lane == 0 && y < H && wi < words) mask[((size_t)plane * H + y) * words + wi] = 0ull;
    }
    TPROF(1, wall_clock64());
  };
  if constexpr (!FUSED) {
    if (bandmax && band_dead(bandmax, plane, H, W, words, y0, x0, thre, &s_live)) {
      zero_masks();
      return;
    }
  } else {
    if (!fused_prologue<WR, WC>(m, nch, plane, H, W, y0, x0, thre, s_low, s_hz, s_ti, s_tb, &s_live)) {
      zero_masks();
      return;
    }
  }
  if (tid == 0) {
    s_live = 0;
    s_amb = 0;
  }
  __syncthreads();
  TPROF(3, clock64());
  // the window: column pair cp (window columns 2cp, 2cp+1) of rows vh*9 .. vh*9+32 (v rows
  // vh*9 .. vh*9+8) per thread, waves 0-1 the first half, 2-3 the second
  const int cp = tid & 127, vh = __builtin_amdgcn_readfirstlane(tid >> 7);   // (wave-uniform)
  const bool vth = cp < NMS_CP;
  f2v a[NMS_VH + 2 * NMS_R];
  if (vth) {
    const int xa = reflect_idx(x0 - 1 - NMS_R + 2 * cp, W), xb = reflect_idx(x0 - NMS_R + 2 * cp, W);
    const T* src = planes + (size_t)plane * H * W;
    double ma = 0.0, mb = 0.0;
    float mfa = 0.f, mfb = 0.f;
    // fused: the 4 stage rows a window row combines (fused_value's taps) move every few rows
    // (strong upsampling), so the column pair's 8 values are re-read from s_hz only when the
    // row's taps change -- the taps are wave-uniform, the branch scalar
    const int rowlen = FUSED ? m.dw * m.cn : 0, fch = FUSED ? plane % nch : 0;
    const bool sva = FUSED && xa * m.cn + fch < rowlen - rowlen % 4;
    const bool svb = FUSED && xb * m.cn + fch < rowlen - rowlen % 4;
    int py0 = -1, py1 = -1, py2 = -1, py3 = -1;
    float ha0 = 0.f, ha1 = 0.f, ha2 = 0.f, ha3 = 0.f, hb0 = 0.f, hb1 = 0.f, hb2 = 0.f, hb3 = 0.f;
#pragma unroll
    for (int k = 0; k < NMS_VH + 2 * NMS_R; ++k) {
      const int r = vh * NMS_VH + k;
      T va, vb;
      if constexpr (!FUSED) {
        // the row is wave-uniform: its reflection and offset are scalar work
        const int rr = y0 - 1 - NMS_R + r;
        const T* row = src + (size_t)((unsigned)rr < (unsigned)H ? rr : reflect_idx(rr, H)) * W;
        va = row[xa];
        vb = row[xb];
      } else {
        const int4 t4 = s_ti[r];
        const int y0t = __builtin_amdgcn_readfirstlane(t4.x), y1t = __builtin_amdgcn_readfirstlane(t4.y);
        const int y2t = __builtin_amdgcn_readfirstlane(t4.z), y3t = __builtin_amdgcn_readfirstlane(t4.w);
        if (y0t != py0 || y1t != py1 || y2t != py2 || y3t != py3) {
          ha0 = s_hz[y0t][2 * cp];
          hb0 = s_hz[y0t][2 * cp + 1];
          ha1 = s_hz[y1t][2 * cp];
          hb1 = s_hz[y1t][2 * cp + 1];
          ha2 = s_hz[y2t][2 * cp];
          hb2 = s_hz[y2t][2 * cp + 1];
          ha3 = s_hz[y3t][2 * cp];
          hb3 = s_hz[y3t][2 * cp + 1];
          py0 = y0t;
          py1 = y1t;
          py2 = y2t;
          py3 = y3t;
        }
        const float4 be = s_tb[r];
        // resize_sep_kernel's vertical combine (VResizeCubicVec_32f body / scalar tail)
        va = sva ? ha0 * be.x + (ha1 * be.y + (ha2 * be.z + ha3 * be.w)) : ((ha0 * be.x + ha1 * be.y) + ha2 * be.z) + ha3 * be.w;
        vb = svb ? hb0 * be.x + (hb1 * be.y + (hb2 * be.z + hb3 * be.w)) : ((hb0 * be.x + hb1 * be.y) + hb2 * be.z) + hb3 * be.w;
      }
      a[k] = f2v{(float)va, (float)vb};
      if constexpr (sizeof(T) == 4) {   // (the max of fp32 magnitudes is exact in fp32)
        mfa = fmaxf(mfa, fabsf((float)va));
        mfb = fmaxf(mfb, fabsf((float)vb));
      } else {
        ma = fmax(ma, fabs((double)va));
        mb = fmax(mb, fabs((double)vb));
      }
      // fp64 planes: at most 11 rows' loads in flight (all 33 pairs of doubles hoisted spill)
      if constexpr (sizeof(T) == 8)
        if (k % 11 == 10) __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (sizeof(T) == 4) {
      ma = (double)mfa;
      mb = (double)mfb;
    }
    s_cmax[vh][2 * cp] = ma;
    s_cmax[vh][2 * cp + 1] = mb;
    // the exact early out (blur_tile_exact): |g| <= max|in| * (1 + 1e-13)
    if (fmax(ma, mb) >= thre * (1.0 - 1e-9)) s_live = 1;
  }
  __syncthreads();
  if (!s_live) {
    zero_masks();
    return;
  }
  TPROF(4, clock64());
  // word liveness (blur_tile_exact's bound per mask word) and M, in wave 0
  if (tid < 64) {
    auto cm = [&](int t) { return fmax(s_cmax[0][t], s_cmax[1][t]); };
    const double ca = cm(tid), cb = cm(64 + tid), cc = cm(128 + tid);
    const double cd = tid < NMS_VC - 192 ? cm(192 + tid) : 0.0;
    double m0 = fmax(ca, tid <= 25 ? cb : 0.0);   // window columns 0..89
    double m1 = fmax(cb, tid <= 25 ? cc : 0.0);   // 64..153
    double m2 = fmax(cc, cd);                     // 128..217
    for (int o = 32; o > 0; o >>= 1) {
      m0 = fmax(m0, __shfl_xor(m0, o));
      m1 = fmax(m1, __shfl_xor(m1, o));
      m2 = fmax(m2, __shfl_xor(m2, o));
    }
    if (tid == 0) {
      s_wlive[0] = m0 >= thre * (1.0 - 1e-9);
      s_wlive[1] = m1 >= thre * (1.0 - 1e-9);
      s_wlive[2] = m2 >= thre * (1.0 - 1e-9);
      s_M = fmax(m0, fmax(m1, m2));
    }
  }
  __syncthreads();
  const bool wl0 = s_wlive[0], wl1 = s_wlive[1], wl2 = s_wlive[2];
  auto col_needed = [&](int t) {
    return (wl0 && t <= 89) || (wl1 && t >= 64 && t <= 153) || (wl2 && t >= 128);
  };
  if (vth && (col_needed(2 * cp) || col_needed(2 * cp + 1))) {
#pragma unroll
    for (int r = 0; r < NMS_VH; ++r) {
      f2v o = a[r + NMS_R] * kGaussF[0];
#pragma unroll
      for (int j = NMS_R; j >= 1; --j)
        o = __builtin_elementwise_fma(a[r + NMS_R - j] + a[r + NMS_R + j], f2v{kGaussF[j], kGaussF[j]}, o);
      *reinterpret_cast<f2v*>(&s_vf[vh * NMS_VH + r][2 * cp]) = o;
    }
  }
  __syncthreads();
  TPROF(5, clock64());
  // horizontal: rows 2p, 2p+1 of g columns c0 .. c0+6 (v columns c0 .. c0+30); g columns
  // c0..c0+6 overlap a live word's g range [64w, 64w+65] (the run's other columns may read v
  // never computed -- their g is never read)
  {
    const int p = tid / NMS_HRUNS, c0 = (tid - p * NMS_HRUNS) * NMS_HSEG, c1 = c0 + NMS_HSEG - 1;
    const bool act = tid < NMS_VR / 2 * NMS_HRUNS &&
                     ((wl0 && c0 <= 65) || (wl1 && c1 >= 64 && c0 <= 129) || (wl2 && c1 >= 128));
    f2v v[NMS_HSEG + 2 * NMS_R];
    if (act) {
#pragma unroll
      for (int k = 0; k < NMS_HSEG + 2 * NMS_R; ++k)
        v[k] = c0 + k < NMS_VC ? f2v{s_vf[2 * p][c0 + k], s_vf[2 * p + 1][c0 + k]} : f2v{0.f, 0.f};
    }
    __syncthreads();   // every v run is in registers: g may overwrite the tile
    if (act) {
#pragma unroll
      for (int k = 0; k < NMS_HSEG; ++k) {
        f2v o = v[k + NMS_R] * kGaussF[0];
#pragma unroll
        for (int j = NMS_R; j >= 1; --j)
          o = __builtin_elementwise_fma(v[k + NMS_R - j] + v[k + NMS_R + j], f2v{kGaussF[j], kGaussF[j]}, o);
        if (c0 + k < NMS_GC) {
          s_vf[2 * p][c0 + k] = o.x;
          s_vf[2 * p + 1][c0 + k] = o.y;
        }
      }
    }
  }
  __syncthreads();
  TPROF(6, clock64());
  // The decisions in fp32: d = fl(g - q) is within 2 u M of g32 - q32 (|g|, |q| <= M) and
  // thre_f = (float)thre within u thre <= u M of thre (a live tile has M >= thre), so with the
  // margin doubled to 2^-17 M (128 u M) the three roundings stay far inside it: "surely" still
  // means the fp64 decision.  (margin_mode 2: M / 4, the re-run of nearly every live tile.)
  const float eps = (float)(s_M * (margin_mode == 2 ? 0.25 : 2.0 * BLUR_EPS_REL)) + 1e-30f, e2 = 2.f * eps;
  const float thre_f = (float)thre;
  // Rows ty = wave, wave+4, .. (wave-uniform), the row's three mask words unrolled: one LDS
  // base per row with immediate offsets, the five reads of a pixel unconditional (rows R-1..R+1,
  // columns cx..cx+2 lie in the tile; behind the plane-edge branches they were serialised LDS
  // round trips), one mask row address per row.
  bool any_open = false;
  for (int ty = wave; ty < NMS_TY; ty += 4) {
    const int y = y0 + ty, R = ty + 1;
    const float* rp = &s_vf[R][lane];
    unsigned long long wv[3];
#pragma unroll
    for (int wd = 0; wd < 3; ++wd) {
      const int cx = wd * 64 + lane, x = x0 + cx;
      const float g = rp[wd * 64 + 1];
      const float fu = rp[wd * 64 + 1 - NMS_VC], fd = rp[wd * 64 + 1 + NMS_VC], fl = rp[wd * 64], fr = rp[wd * 64 + 2];
      // (branch-free in the neighbours, so that the five reads are not sunk behind a branch)
      const float dt = g - thre_f;
      const float d0 = g - (y > 0 ? fu : 0.f), d1 = g - (y + 1 < H ? fd : 0.f);
      const float d2 = g - (x > 0 ? fl : 0.f), d3 = g - (x + 1 < W ? fr : 0.f);
      const float dmin = fminf(fminf(d0, d1), fminf(d2, d3));   // (no NaN: finite planes)
      const bool nb = !mode_hand;
      // surely g < thre, or surely g < a neighbour (the pixel is out)
      const bool no = dt <= -eps || (nb && dmin < -e2);
      // g vs thre, or g vs a neighbour, inside the margin
      const bool inm = !(dt > eps) || (nb && !(dmin >= e2));
      const bool valid = y < H && x < W && (wd == 0 ? wl0 : wd == 1 ? wl1 : wl2);
      const bool pk = valid && !no && !inm;
      const bool open = valid && !no && inm;
      wv[wd] = __ballot(pk);
      any_open = any_open || __ballot(open) != 0;
    }
    if (lane == 0 && y < H) {
      unsigned long long* mrow = mask + ((size_t)plane * H + y) * words + bx * 3;
#pragma unroll
      for (int wd = 0; wd < 3; ++wd)
        if (bx * 3 + wd < words) mrow[wd] = wv[wd];
    }
  }
  if (lane == 0 && any_open) s_amb = 1;
  __syncthreads();
  TPROF(7, clock64());
  TPROF(1, wall_clock64());
  if (tid == 0 && s_amb) {
    amb[atomicAdd(amb_count, 1)] = tile_id;   // the exact passes re-run the whole tile
    TPROF(8, 1);
  }
}

// One tile per block (live == nullptr: the grid is tiles_x x tiles_y x planes), or a
// grid-stride loop over a list of tiles (tile_live_kernel / band_live_kernel / the filter's
// undecided tiles; the mask pre-zeroed where a list skips tiles).  EXACT: the fp64 passes;
// else the fp32 filter, appending undecided tiles to amb.
// (4 waves per SIMD: the register allocation is held to that occupancy, 128 VGPRs; the
// filter on fp64 planes -- the multi-scale and hand averages -- 3 waves, 168 VGPRs, unspilled)
template <typename T, bool FUSED, bool EXACT, int WR = NMS_SRC_ROWS, int WC = NMS_SRC_COLS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 8 && !EXACT ? 3 : 4)))
    blur_nms_kernel(const T* __restrict__ planes, int H, int W, int words, unsigned long long* __restrict__ mask,
                    double thre, int mode_hand, MapSrc m, int nch, const int* __restrict__ live,
                    const int* __restrict__ live_count, int tiles_x, int tiles_y, const float* __restrict__ bandmax,
                    int* __restrict__ amb, int* __restrict__ amb_count, int margin_mode) {
  auto run = [&](int plane, int by, int bx) {
    if constexpr (EXACT)
      blur_tile_exact<T, FUSED, WR, WC>(planes, H, W, words, mask, thre, mode_hand, m, nch, plane, by, bx, bandmax);
    else
      blur_tile_filter<T, FUSED, WR, WC>(planes, H, W, words, mask, thre, mode_hand, m, nch, plane, by, bx, bandmax,
                                         amb, amb_count, (plane * tiles_y + by) * tiles_x + bx, margin_mode);
  };
  if (!live) {
    run(blockIdx.z, blockIdx.y, blockIdx.x);
  } else {
    // XCD-aware: workgroups land on the 8 XCDs round-robin, so XCD x takes the x-th eighth of
    // the (roughly tile-ordered) list -- neighbouring tiles, whose windows share 26 of 42 rows,
    // then meet in one L2 (any placement is correct; a grid that is not a multiple of 8 strides)
    const int cnt = *live_count;
    constexpr int NX = 8;
    const bool part = gridDim.x % NX == 0;
    const int xcd = part ? blockIdx.x % NX : 0, per = part ? gridDim.x / NX : gridDim.x;
    const int k0 = part ? (int)((long long)cnt * xcd / NX) : 0;
    const int k1 = part ? (int)((long long)cnt * (xcd + 1) / NX) : cnt;
    for (int k = k0 + (part ? blockIdx.x / NX : blockIdx.x); k < k1; k += per) {
      const int t = live[k];
      const int bx = t % tiles_x, r = t / tiles_x, by = r % tiles_y, plane = r / tiles_y;
      run(plane, by, bx);
      __syncthreads();   // LDS reuse by the next tile
    }
  }
}

// ISLPOSE_BLUR_EXACT=1: every live tile on the fp64 passes, without the fp32 filter; =2: the
// filter with a margin so wide that nearly every live tile falls back (A/B and the filter's
// tests: the same mask bits either way; per call)
static int blur_exact_only() {
  const char* e = getenv("ISLPOSE_BLUR_EXACT");
  return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
}

// The blur of one post: the filter launch, then the exact passes over the tiles it could
// not decide (a grid-stride launch over its list; ISLPOSE_BLUR_EXACT=1: the exact passes
// over every tile instead).  `grid` / `live`: one tile per block or a live list (as
// blur_nms_kernel); amb: n_tiles + 1 ints of scratch.
template <typename T, bool FUSED, int WR = NMS_SRC_ROWS, int WC = NMS_SRC_COLS>
static int launch_blur(dim3 grid, hipStream_t s, const T* planes, int H, int W, int words, unsigned long long* mask,
                       double thre, int mode_hand, const MapSrc& m, int nch, const int* live, const int* live_count,
                       int tiles_x, int tiles_y, const float* bandmax, int* amb, bool amb_zeroed = false) {
  const int ex = blur_exact_only();
  if (ex == 1) {
    hipLaunchKernelGGL((blur_nms_kernel<T, FUSED, true, WR, WC>), grid, dim3(256), 0, s, planes, H, W, words, mask,
                       thre, mode_hand, m, nch, live, live_count, tiles_x, tiles_y, bandmax, nullptr, nullptr, 0);
    return hipGetLastError() == hipSuccess ? ISL_OK : ISL_E_HIP;
  }
  int* amb_count = amb;
  if (!amb_zeroed && hipMemsetAsync(amb_count, 0, sizeof(int), s) != hipSuccess) return ISL_E_HIP;
  hipLaunchKernelGGL((blur_nms_kernel<T, FUSED, false, WR, WC>), grid, dim3(256), 0, s, planes, H, W, words, mask,
                     thre, mode_hand, m, nch, live, live_count, tiles_x, tiles_y, bandmax, amb + 1, amb_count, ex);
  if (hipGetLastError() != hipSuccess) return ISL_E_HIP;
  hipLaunchKernelGGL((blur_nms_kernel<T, FUSED, true, WR, WC>), dim3(256), dim3(256), 0, s, planes, H, W, words, mask,
                     thre, mode_hand, m, nch, (const int*)(amb + 1), (const int*)amb_count, tiles_x, tiles_y,
                     (const float*)nullptr, nullptr, nullptr, 0);
  return hipGetLastError() == hipSuccess ? ISL_OK : ISL_E_HIP;
}

// Two-stage single-scale frames (Mode R: the net's valid crop -> stage 1 -> stage 2 to the frame):
// which blur tiles can be live at all, from the stage-1 planes' band maxima (bm1: 16-row bands
// x 64-column words, resize_sep_kernel BM), and which stage-2 resize tiles (rows ty2 x 128
// columns) their windows read.  |stage-2 value| <= 1.890625 max|stage-1 value| over its 4 x 4
// taps (the cubic weights' absolute sums, squared), fp32 rounding inside the 1.9 factor
// (blur_tile's fused bound), so a tile whose window's stage-1 source stays below thre / 1.9 is
// dead; every tile a live window overlaps is marked in `need` (zeroed by the caller).
__global__ void __launch_bounds__(256) stage2_need_kernel(MapSrc m2, const float* __restrict__ bm1, int H, int W,
                                                          int tiles_x, int tiles_y, int n_tiles, double thre, int ty2,
                                                          int ry_tiles, int rx_tiles, unsigned char* __restrict__ live_mid,
                                                          unsigned char* __restrict__ need) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n_tiles) return;
  const int bx = t % tiles_x, r = t / tiles_x, by = r % tiles_y, plane = r / tiles_y;
  const int y0 = by * NMS_TY, x0 = bx * NMS_TX;
  int rlo, rhi, clo, chi;
  reflect_range(y0 - 1 - NMS_R, y0 - 2 - NMS_R + NMS_IR, H, &rlo, &rhi);
  reflect_range(x0 - 1 - NMS_R, x0 - 2 - NMS_R + NMS_VC, W, &clo, &chi);
  int a[4], b[4];
  float dmy[4];
  taps(rlo, m2.scy, m2.sh, a, dmy);
  taps(rhi, m2.scy, m2.sh, b, dmy);
  const int mb0 = a[0] / BM_ROWS, mb1 = b[3] / BM_ROWS;
  taps(clo, m2.scx, m2.sw, a, dmy);
  taps(chi, m2.scx, m2.sw, b, dmy);
  const int mw0 = a[0] / 64, mw1 = b[3] / 64;
  const int bands1 = (m2.sh + BM_ROWS - 1) / BM_ROWS, words1 = (m2.sw + 63) / 64;
  float mx = 0.f;
  for (int i = mb0; i <= mb1; ++i)
    for (int j = mw0; j <= mw1; ++j) mx = fmaxf(mx, bm1[((size_t)plane * bands1 + i) * words1 + j]);
  const bool lv = (double)mx * 1.9 >= thre * (1.0 - 1e-9);
  live_mid[t] = lv;
  if (lv)
    for (int ry = rlo / ty2; ry <= rhi / ty2; ++ry)
      for (int rx = clo / 128; rx <= chi / 128; ++rx) need[((size_t)plane * ry_tiles + ry) * rx_tiles + rx] = 1;
}

// The band-maxima bound of the materialised single-scale path, one tile per thread: the
// tile's window, reflected, against resize_sep_kernel's band x word maxima (blur_tile's own
// early out, before any block is launched for the tile); live tiles are appended to `live`
// (one atomic per wave).  The blur then runs over the live tiles only (mask pre-zeroed).
__global__ void __launch_bounds__(256) band_live_kernel(const float* __restrict__ bandmax, int H, int W, int words,
                                                        int tiles_x, int tiles_y, int n_tiles, double thre,
                                                        int* __restrict__ live, int* __restrict__ live_count,
                                                        const unsigned char* __restrict__ live_mid = nullptr) {
  const int t = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
  int lv = 0;
  if (t < n_tiles && (!live_mid || live_mid[t])) {   // (stage-2 tiles of a dead window were skipped)
    const int bx = t % tiles_x, r = t / tiles_x, by = r % tiles_y, plane = r / tiles_y;
    const int y0 = by * NMS_TY, x0 = bx * NMS_TX;
    int rlo, rhi, clo, chi;
    reflect_range(y0 - 1 - NMS_R, y0 - 2 - NMS_R + NMS_IR, H, &rlo, &rhi);
    reflect_range(x0 - 1 - NMS_R, x0 - 2 - NMS_R + NMS_VC, W, &clo, &chi);
    const int b0 = rlo / BM_ROWS, nb = rhi / BM_ROWS - b0 + 1, w0 = clo / 64, nw = chi / 64 - w0 + 1;
    const int bands = (H + BM_ROWS - 1) / BM_ROWS;
    if (nb * nw > 64) {
      lv = 1;                                   // (tiny planes: no early out, as blur_tile)
    } else {
      float mx = 0.f;
      for (int i = 0; i < nb; ++i)
        for (int j = 0; j < nw; ++j) mx = fmaxf(mx, bandmax[((size_t)plane * bands + b0 + i) * words + w0 + j]);
      lv = (double)mx >= thre * (1.0 - 1e-9);
    }
  }
  const unsigned long long bal = __ballot(lv);
  int base = 0;
  if (lane == 0 && bal) base = atomicAdd(live_count, (int)__popcll(bal));
  base = __shfl(base, 0);
  if (lv) live[base + __popcll(bal & ((1ull << lane) - 1))] = t;
}

// The low-res bound of the fused path for TL_TILES consecutive blur tiles per block
// (one wave per tile at a time); live tiles are appended to `live` with one atomic
// per block (order irrelevant: every tile owns its mask words).
constexpr int TL_TILES = 16;   // 4 tiles per wave: enough blocks to hide the load latency
template <int WR, int WC>
__global__ void __launch_bounds__(256) tile_live_kernel(MapSrc m, int nch, int H, int W, int tiles_x, int tiles_y,
                                                        int n_tiles, double thre, int* __restrict__ live,
                                                        int* __restrict__ live_count) {
  __shared__ int s_flag[TL_TILES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int j = wave; j < TL_TILES; j += 4) {
    const int t = blockIdx.x * TL_TILES + j;
    int live_t = 0;
    if (t < n_tiles) {
      const int bx = t % tiles_x, r = t / tiles_x, by = r % tiles_y, plane = r / tiles_y;
      const int f = plane / nch, c = plane - f * nch;
      const float* b = m.base + (size_t)f * m.fs + chan_off(m, c);
      int sr0, nsr, sc0, nsc;
      fused_window(m, H, W, by * NMS_TY, bx * NMS_TX, &sr0, &nsr, &sc0, &nsc);
      float amax = 0.f;
      if (nsr > WR || nsc > WC) __builtin_trap();   // the host picks a window that holds them
      for (int cc = lane; cc < nsc; cc += 64) {   // one column per lane, all rows in flight
        const float* col = b + (size_t)(sc0 + cc) * m.xs + (size_t)sr0 * m.ys;
#pragma unroll
        for (int rr = 0; rr < WR; ++rr)
          if (rr < nsr) amax = fmaxf(amax, fabsf(col[(size_t)rr * m.ys]));
      }
      for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
      live_t = (double)amax * 1.9 >= thre * (1.0 - 1e-9);
    }
    if (lane == 0) s_flag[j] = live_t;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    static_assert(TL_TILES <= 64, "one wave publishes the block's flags");
    const int fl = lane < TL_TILES ? s_flag[lane] : 0;
    const unsigned long long bal = __ballot(fl);
    int base = 0;
    if (lane == 0 && bal) base = atomicAdd(live_count, (int)__popcll(bal));
    base = __shfl(base, 0);
    if (fl) live[base + __popcll(bal & ((1ull << lane) - 1))] = blockIdx.x * TL_TILES + lane;
  }
}

// ---------------------------------------------------------------------------
// peak compaction: np.nonzero (row-major) order, one block per (frame, part)
// ---------------------------------------------------------------------------

// FUSED: scores sampled from the low-res map with the resize's arithmetic (the
// full-resolution plane was never written; blur_nms_kernel<float, true>)
template <typename T, bool FUSED>
__global__ void __launch_bounds__(256) compact_kernel(const unsigned long long* __restrict__ mask,
                                                       const T* __restrict__ planes, int nparts, int H, int W,
                                                       int words, char* __restrict__ result, isl_layout lay,
                                                       int max_peaks, MapSrc m) {
  const int f = blockIdx.y, part = blockIdx.x;
  const int plane = f * nparts + part;
  const unsigned long long* mk = mask + (size_t)plane * H * words;
  const T* src = planes + (size_t)plane * H * W;
  char* rec = result + (size_t)f * lay.record_bytes;
  double* peaks = (double*)(rec + lay.peaks) + (size_t)part * max_peaks * 3;
  // Raster order (np.nonzero): each thread owns CW consecutive words of a round, its peaks
  // go after those of the lower threads (a wave prefix by shuffles, the four wave totals in
  // LDS), rounds in order.  (The 256-wide Hillis-Steele scan of 1024 words per round was 16
  // barriers per round: 57 us per 1080p frame of mostly empty rounds, profiles/r06/lk/.)
  constexpr int CW = 8;
  __shared__ int s_w[4];
  __shared__ int s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nw = H * words;
  if (tid == 0) s_base = 0;
  __syncthreads();
  for (int w0 = 0; w0 < nw; w0 += 256 * CW) {
    unsigned long long wv[CW];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < CW; ++k) {
      const int wi = w0 + tid * CW + k;
      wv[k] = wi < nw ? mk[wi] : 0ull;
      cnt += __popcll(wv[k]);
    }
    int inc = cnt;   // inclusive prefix over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(inc, d, 64);
      if (lane >= d) inc += y;
    }
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    int pos = s_base + inc - cnt;
    for (int q = 0; q < wave; ++q) pos += s_w[q];
    const int round_total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    if (cnt) {
#pragma unroll
      for (int k = 0; k < CW; ++k) {
        const int wi = w0 + tid * CW + k;
        unsigned long long w = wv[k];
        while (w) {
          const int b = __ffsll((long long)w) - 1;
          w &= w - 1;
          const int y = wi / words, x = (wi - y * words) * 64 + b;
          if (pos < max_peaks) {
            double* p = peaks + (size_t)pos * 3;
            p[0] = (double)x;
            p[1] = (double)y;
            if constexpr (FUSED) p[2] = (double)sample(m, f, part, y, x);
            else p[2] = (double)src[(size_t)y * W + x];
          }
          ++pos;
        }
      }
    }
    __syncthreads();   // every thread has read s_base and s_w
    if (tid == 0) s_base += round_total;
    __syncthreads();
  }
  if (tid == 0) {
    ((int*)(rec + lay.n_peaks))[part] = s_base;
    if (s_base > max_peaks) atomicExch((int*)(rec + lay.status), ISL_E_CAPACITY);
  }
}

// ---------------------------------------------------------------------------
// PAF scoring + greedy matching + assembly (body.py:128-235), one block per frame
// ---------------------------------------------------------------------------

constexpr int MAX_SCALES = 8;
static_assert(sizeof(MapSrcN::m) / sizeof(MapSrc) == MAX_SCALES, "resize_acc_kernel takes every scale");

struct GroupArgs {
  MapSrc paf[MAX_SCALES];   // final-resolution PAF of each scale (sampled on demand)
  MapSrc paf1[MAX_SCALES];  // nested scales: the stage-1 resize that paf[s] reads, never materialised
  int paf_nested[MAX_SCALES];
  int nscales;
  float div_f;              // len(multiplier), as float32
  int H, W;                 // frame size
  int model;                // ISL_BODY25 / ISL_COCO
  int njoint, nlimbs;
  int max_peaks, max_pairs, max_conns, max_rows;
  isl_layout lay;
  char* result;
  double* pair_score;       // [n][max_pairs]
  int* pair_keep;           // [n][max_pairs]  (-1 rejected, else rank key)
  int* order;               // [n][max_pairs]
  unsigned char* used;      // [n][2][max_peaks]
  int limb_lds;             // large pair sets ranked in LDS (ISLPOSE_LIMB_LDS=0: the per-thread pair loop)
};

// One element of the two-stage resize m2(m1(low)) (body.py:68-73 then :74-76 on a frame whose
// net input is not the frame) without the stage-1 planes: the 4 x 4 stage-1 values the
// stage-2 taps read, each exactly as resize_sep_kernel computes it (sample()'s order), with
// the stage-1 horizontal combinations of the <= 5 low-resolution rows they span shared.
__device__ float sample_nested(const MapSrc& m2, const MapSrc& m1, int f, int c, int y, int x) {
  int xi[4], yi[4];
  float a[4], be[4];
  taps(x, m2.scx, m2.sw, xi, a);
  taps(y, m2.scy, m2.sh, yi, be);
  const float* b = m1.base + (size_t)f * m1.fs + chan_off(m1, c);
  int lxi[4][4], lyi[4][4];
  float la[4][4], lbe[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    taps(xi[k], m1.scx, m1.sw, lxi[k], la[k]);
    taps(yi[k], m1.scy, m1.sh, lyi[k], lbe[k]);
  }
  const int r0 = lyi[0][0];   // taps are monotone in the index: rows r0 .. lyi[3][3]
  const int rowlen1 = m1.dw * m1.cn;
  float s1[4][4];
  if (lyi[3][3] - r0 < 5) {
    float h1[5][4];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const float* row = b + (size_t)min(r0 + r, lyi[3][3]) * m1.ys;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        h1[r][k] = ((row[lxi[k][0] * m1.xs] * la[k][0] + row[lxi[k][1] * m1.xs] * la[k][1]) +
                    row[lxi[k][2] * m1.xs] * la[k][2]) + row[lxi[k][3] * m1.xs] * la[k][3];
    }
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        float h[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int r = lyi[ky][t] - r0;   // 0..4: a select chain, no private array
          h[t] = r == 0 ? h1[0][kx] : r == 1 ? h1[1][kx] : r == 2 ? h1[2][kx] : r == 3 ? h1[3][kx] : h1[4][kx];
        }
        const float* bb = lbe[ky];
        s1[ky][kx] = xi[kx] * m1.cn + c < rowlen1 - rowlen1 % 4
                         ? h[0] * bb[0] + (h[1] * bb[1] + (h[2] * bb[2] + h[3] * bb[3]))
                         : ((h[0] * bb[0] + h[1] * bb[1]) + h[2] * bb[2]) + h[3] * bb[3];
      }
    }
  } else {
#pragma unroll
    for (int ky = 0; ky < 4; ++ky)
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) s1[ky][kx] = sample_row(m1, f, c, lyi[ky], lbe[ky], xi[kx]);
  }
  float hz[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) hz[k] = ((s1[k][0] * a[0] + s1[k][1] * a[1]) + s1[k][2] * a[2]) + s1[k][3] * a[3];
  const int rowlen = m2.dw * m2.cn;
  if (x * m2.cn + c < rowlen - rowlen % 4) return hz[0] * be[0] + (hz[1] * be[1] + (hz[2] * be[2] + hz[3] * be[3]));
  return ((hz[0] * be[0] + hz[1] * be[1]) + hz[2] * be[2]) + hz[3] * be[3];
}

__device__ __forceinline__ double paf_value(const GroupArgs& a, int f, int c, int y, int x) {
  double acc = 0.0;
  for (int s = 0; s < a.nscales; ++s) {
    const float v = a.paf_nested[s] ? sample_nested(a.paf[s], a.paf1[s], f, c, y, x) : sample(a.paf[s], f, c, y, x);
    acc = acc + (double)(v / a.div_f);   // paf_avg += + paf / len(multiplier)
  }
  return acc;
}

constexpr int LIMB_ITEMS = 2048;   // (pair, point) items scored in parallel (16 KB of LDS)
constexpr int LIMB_MAXP = 4096;    // large pair sets ranked and matched in LDS (the default max_pairs)
constexpr int LIMB_MAXPK = 1024;   // ... with at most this many peaks of either part (used flags in LDS)
// One workgroup per (limb, frame): score every (A, B) pair (body.py:142-164),
// stable descending sort by rank counting, greedy matching (body.py:166-175).
// MODE 0: all of it.  Small batches (a frame per call) spread the scoring, the bulk of the work
// (two nested PAF samples per (pair, point)), over more CUs: MODE 1 blocks (limb, frame, z)
// score the z-th slice of a limb's pairs into pscore / pkeep, then MODE 2 (one block per limb
// and frame) ranks and matches them.  The same sums in the same order: the same scores.
// (3 waves per SIMD: the inlined nested samples took 212 VGPRs, 2 waves per SIMD, and a batch-32
// grid of 832 blocks ran in two rounds; at 168 VGPRs the spills sit in the large-set path:
// Mode R batch 32 44.6 -> 38.8 us, profiles/r05/r5lb)
template <int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) limb_kernel(GroupArgs a) {
  const int k = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  char* rec = a.result + (size_t)f * a.lay.record_bytes;
  int* status = (int*)(rec + a.lay.status);
  const int* n_peaks = (const int*)(rec + a.lay.n_peaks);
  int* n_conns = (int*)(rec + a.lay.n_conns);
  const double* peaks = (const double*)(rec + a.lay.peaks);
  double* conns = (double*)(rec + a.lay.conns);
  const size_t slot = (size_t)f * a.nlimbs + k;
  double* pscore = a.pair_score + slot * a.max_pairs;
  int* pkeep = a.pair_keep + slot * a.max_pairs;
  int* order = a.order + slot * a.max_pairs;
  unsigned char* usedA = a.used + slot * 2 * a.max_peaks;
  unsigned char* usedB = usedA + a.max_peaks;
  __shared__ int s_offA, s_offB, s_nkeep;
  __shared__ double s_item[LIMB_ITEMS];
  if (*status != ISL_OK) return;    // capacity overflow in compaction: host re-runs with larger caps
  const int A = a.model == ISL_BODY25 ? kLimbs25[k][0] : kLimbsCoco[k][0];
  const int B = a.model == ISL_BODY25 ? kLimbs25[k][1] : kLimbsCoco[k][1];
  const int mx = a.model == ISL_BODY25 ? kMap25[k][0] : kMapCoco[k][0];
  const int my = a.model == ISL_BODY25 ? kMap25[k][1] : kMapCoco[k][1];
  const int nA = n_peaks[A], nB = n_peaks[B];
  if (nA == 0 || nB == 0) {            // special_k
    if (MODE != 1 && tid == 0) n_conns[k] = -1;
    return;
  }
  const int np = nA * nB;
  if (np > a.max_pairs) {
    if (MODE != 1 && tid == 0) { atomicExch(status, ISL_E_CAPACITY); n_conns[k] = -2; }
    return;
  }
  if (tid == 0) {
    int acc = 0;
    for (int p = 0; p < a.njoint - 1; ++p) {
      if (p == A) s_offA = acc;
      if (p == B) s_offB = acc;
      acc += n_peaks[p];
    }
    s_nkeep = 0;
  }
  const double* pA = peaks + (size_t)A * a.max_peaks * 3;
  const double* pB = peaks + (size_t)B * a.max_peaks * 3;
  // pair p's direction, norm and sample point I (np.linspace, int(round(.)): half to even)
  auto point = [&](int p, int I, double* ux, double* uy, double* norm, int* xi, int* yi) {
    const int i = p / nB, j = p - i * nB;
    const long long ax = (long long)pA[i * 3], ay = (long long)pA[i * 3 + 1];
    const long long bx = (long long)pB[j * 3], by = (long long)pB[j * 3 + 1];
    const long long vx = bx - ax, vy = by - ay;
    double nr = sqrt((double)(vx * vx + vy * vy));       // math.sqrt of an exact integer
    nr = 0.001 < nr ? nr : 0.001;                         // max(0.001, norm)
    *norm = nr;
    *ux = (double)vx / nr;
    *uy = (double)vy / nr;
    const double stx = ((double)bx - (double)ax) / 9.0, sty = ((double)by - (double)ay) / 9.0;
    const double sx = I == 9 ? (double)bx : (double)I * stx + (double)ax;
    const double sy = I == 9 ? (double)by : (double)I * sty + (double)ay;
    *xi = (int)rint(sx);
    *yi = (int)rint(sy);
  };
  auto score_val = [&](double sum, double norm) {
    const double prior = 0.5 * (double)a.H / norm - 1.0;
    return sum / 10.0 + (0.0 < prior ? 0.0 : prior);
  };
  auto score_of = [&](int p, double sum, int cnt, double norm) {
    const double score = score_val(sum, norm);
    pscore[p] = score;
    pkeep[p] = (cnt > 8 && score > 0.0) ? 1 : 0;
  };
  // pairs [q0, q1): their (pair, point) items in chunks of LIMB_ITEMS / 20 pairs, the two PAF
  // channels of a point on two threads (products added in order after the barrier, as the small
  // path), each pair's sum in point order into pscore / pkeep
  auto score_range = [&](int q0, int q1) __attribute__((always_inline)) {
    constexpr int CP = LIMB_ITEMS / 20;
    for (int p0 = q0; p0 < q1; p0 += CP) {
      const int pc = min(CP, q1 - p0);
      for (int it = tid; it < pc * 20; it += 256) {
        const int item = it >> 1, ch = it & 1;
        double ux, uy, nr;
        int xi, yi;
        point(p0 + item / 10, item % 10, &ux, &uy, &nr, &xi, &yi);
        s_item[it] = paf_value(a, f, ch ? my : mx, yi, xi) * (ch ? uy : ux);
      }
      __syncthreads();
      for (int q = tid; q < pc; q += 256) {
        double sum = 0.0;
        int cnt = 0;
        for (int I = 0; I < 10; ++I) {
          const double v = s_item[(q * 10 + I) * 2] + s_item[(q * 10 + I) * 2 + 1];
          sum = sum + v;                                                      // builtin sum(), left to right
          cnt += v > 0.05;
        }
        double ux, uy, nr;
        int xi, yi;
        point(p0 + q, 0, &ux, &uy, &nr, &xi, &yi);
        score_of(p0 + q, sum, cnt, nr);
      }
      __syncthreads();   // s_item is reused
    }
  };
  if constexpr (MODE == 1) {
    const int Z = gridDim.z, per = (np + Z - 1) / Z;
    const int q0 = min(np, (int)blockIdx.z * per), q1 = min(np, q0 + per);
    score_range(q0, q1);
    return;
  }
  if (np * 10 <= LIMB_ITEMS) {
    // every (pair, point) in parallel (the nested two-stage samples are ~80 loads each), then
    // each pair's sum in point order
    // small pair sets (np * 20 <= LIMB_ITEMS: a batch-1 frame's limbs) take the two PAF channels
    // of a point on two threads, so a thread's chain is one sample; the products are added in the
    // same order after the barrier (vx * ux + vy * uy)
    const bool split = np * 20 <= LIMB_ITEMS;
    if (MODE == 2) {
      // scored by the MODE 1 launch
    } else if (split) {
      for (int it = tid; it < np * 20; it += 256) {
        const int item = it >> 1, ch = it & 1;
        double ux, uy, nr;
        int xi, yi;
        point(item / 10, item % 10, &ux, &uy, &nr, &xi, &yi);
        s_item[it] = paf_value(a, f, ch ? my : mx, yi, xi) * (ch ? uy : ux);
      }
      __syncthreads();
      double sv[LIMB_ITEMS / 2 / 256 + 1];
      int nv = 0;
      for (int it = tid; it < np * 10; it += 256) sv[nv++] = s_item[2 * it] + s_item[2 * it + 1];
      __syncthreads();
      nv = 0;
      for (int it = tid; it < np * 10; it += 256) s_item[it] = sv[nv++];
    } else {
      for (int it = tid; it < np * 10; it += 256) {
        double ux, uy, nr;
        int xi, yi;
        point(it / 10, it % 10, &ux, &uy, &nr, &xi, &yi);
        s_item[it] = paf_value(a, f, mx, yi, xi) * ux + paf_value(a, f, my, yi, xi) * uy;
      }
    }
    // (these pairs' scores, keep flags, rank order and used flags live in LDS: the rank sort and
    // the serial greedy below then wait on no global load)
    __shared__ double s_ps[LIMB_ITEMS / 10];
    __shared__ int s_pk[LIMB_ITEMS / 10], s_or[LIMB_ITEMS / 10];
    __shared__ unsigned char s_ua[LIMB_ITEMS / 10], s_ub[LIMB_ITEMS / 10];
    __syncthreads();
    for (int p = tid; p < np; p += 256) {
      if (MODE == 2) {
        s_ps[p] = pscore[p];
        s_pk[p] = pkeep[p];
        continue;
      }
      double sum = 0.0;
      int cnt = 0;
      for (int I = 0; I < 10; ++I) {
        const double s = s_item[p * 10 + I];
        sum = sum + s;                                                        // builtin sum(), left to right
        cnt += s > 0.05;
      }
      double ux, uy, nr;
      int xi, yi;
      point(p, 0, &ux, &uy, &nr, &xi, &yi);
      const double score = score_val(sum, nr);
      s_ps[p] = score;
      s_pk[p] = (cnt > 8 && score > 0.0) ? 1 : 0;
    }
    for (int i = tid; i < nA; i += 256) s_ua[i] = 0;   // (nA, nB <= np <= LIMB_ITEMS / 10)
    for (int j = tid; j < nB; j += 256) s_ub[j] = 0;
    __syncthreads();
    // stable descending sort of the kept pairs (sorted(..., reverse=True)): rank = #(better)
    for (int p = tid; p < np; p += 256) {
      if (!s_pk[p]) continue;
      const double sp = s_ps[p];
      int rank = 0;
      for (int q = 0; q < np; ++q)
        if (s_pk[q] && (s_ps[q] > sp || (s_ps[q] == sp && q < p))) ++rank;
      s_or[rank] = p;
      atomicAdd(&s_nkeep, 1);
    }
    __syncthreads();
    if (tid == 0) {
      double* cw = conns + (size_t)k * a.max_conns * 5;
      const int lim = nA < nB ? nA : nB;
      int m = 0;
      for (int r = 0; r < s_nkeep && m < lim; ++r) {
        const int p = s_or[r];
        const int i = p / nB, j = p - i * nB;
        if (s_ua[i] || s_ub[j]) continue;
        s_ua[i] = s_ub[j] = 1;
        if (m >= a.max_conns) { atomicExch(status, ISL_E_CAPACITY); break; }
        double* c = cw + (size_t)m * 5;
        c[0] = (double)(s_offA + i);
        c[1] = (double)(s_offB + j);
        c[2] = s_ps[p];
        c[3] = (double)i;
        c[4] = (double)j;
        ++m;
      }
      n_conns[k] = m;
    }
    return;
  } else if (a.limb_lds && np <= LIMB_MAXP && nA <= LIMB_MAXPK && nB <= LIMB_MAXPK) {
    // Large pair sets (crowded or noisy frames: a 1080p frame's limbs reach hundreds of pairs).
    // The (pair, point) items in chunks of LIMB_ITEMS / 10 pairs, every thread at once, each
    // pair's sum in point order into pscore / pkeep; the rank sort over LDS tiles of the kept
    // scores (a thread's pairs counted against each staged score); the order, the sorted scores
    // and the used flags in LDS for the serial greedy.  Same sums, ranks and matches as the
    // per-thread pair loop below, which walked dependent global loads in its O(np^2) rank sort
    // and its greedy (~0.9 ms per 1080p frame).
    if (MODE == 0) score_range(0, np);
    __shared__ int s_ord[LIMB_MAXP];
    __shared__ unsigned char s_uA[LIMB_MAXPK], s_uB[LIMB_MAXPK];
    // The stable descending sort (sorted(..., reverse=True)) as a bitonic sort in LDS on (score,
    // pair): a before b iff score_a > score_b or (equal and a < b) -- a strict total order, so the
    // permutation the rank count gave.  Pairs not kept (and the padding to a power of two) sort
    // last as -inf.  (The rank count, O(np^2 / 256) per thread: limb scoring 215 us per 1080p
    // frame, profiles/r06/lk1/.)
    __shared__ double s_key[LIMB_MAXP];
    int N = 2;
    while (N < np) N <<= 1;
    __syncthreads();   // s_nkeep zeroed
    for (int i = tid; i < N; i += 256) {
      const bool kept = i < np && pkeep[i];
      s_key[i] = kept ? pscore[i] : -INFINITY;
      s_ord[i] = i;
      if (kept) atomicAdd(&s_nkeep, 1);
    }
    __syncthreads();
    for (int size = 2; size <= N; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = tid; t < N / 2; t += 256) {
          const int i = 2 * t - (t & (stride - 1)), j = i + stride;
          const double ki = s_key[i], kj = s_key[j];
          const int oi = s_ord[i], oj = s_ord[j];
          const bool j_first = kj > ki || (kj == ki && oj < oi);
          if (((i & size) == 0) == j_first) {   // (i & size) == 0: this run sorts first-to-last
            s_key[i] = kj; s_key[j] = ki;
            s_ord[i] = oj; s_ord[j] = oi;
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < nA; i += 256) s_uA[i] = 0;
    for (int j = tid; j < nB; j += 256) s_uB[j] = 0;
    __syncthreads();
    // The greedy (body.py:166-175) on wave 0, 64 sorted pairs at a time: every lane loads its
    // pair and drops it if an endpoint is already used; the survivors are then taken in order
    // by the whole wave (lowest lane first), each re-checked against the pairs accepted before
    // it in this batch.  The same accepts in the same order as one thread walking the list.
    if ((tid >> 6) == 0) {
      const int lane = tid & 63;
      volatile unsigned char* uA = s_uA;
      volatile unsigned char* uB = s_uB;
      double* cw = conns + (size_t)k * a.max_conns * 5;
      const int lim = nA < nB ? nA : nB, nkeep = s_nkeep;
      int m = 0;
      bool full = false;
      for (int r0 = 0; r0 < nkeep && m < lim && !full; r0 += 64) {
        const int r = r0 + lane;
        int i = 0, j = 0;
        bool cand = false;
        if (r < nkeep) {
          const int p = s_ord[r];
          i = p / nB;
          j = p - i * nB;
          cand = !uA[i] && !uB[j];
        }
        unsigned long long live = __ballot(cand);
        while (live && m < lim) {
          const int l = __builtin_ctzll(live);
          live &= live - 1;
          const int il = __shfl(i, l, 64), jl = __shfl(j, l, 64);
          if (uA[il] || uB[jl]) continue;          // taken by an earlier pair of this batch
          if (m >= a.max_conns) {
            if (lane == 0) atomicExch(status, ISL_E_CAPACITY);
            full = true;
            break;
          }
          if (lane == 0) {
            uA[il] = 1;
            uB[jl] = 1;
          }
          if (lane < 5) {
            double* c = cw + (size_t)m * 5;
            c[lane] = lane == 0 ? (double)(s_offA + il) : lane == 1 ? (double)(s_offB + jl)
                    : lane == 2 ? s_key[r0 + l] : lane == 3 ? (double)il : (double)jl;
          }
          ++m;
        }
      }
      if (lane == 0) n_conns[k] = m;
    }
    return;
  } else if (MODE == 0) {
    for (int p = tid; p < np; p += 256) {
      double sum = 0.0, nr = 0.0;
      int cnt = 0;
      for (int I = 0; I < 10; ++I) {
        double ux, uy;
        int xi, yi;
        point(p, I, &ux, &uy, &nr, &xi, &yi);
        const double s = paf_value(a, f, mx, yi, xi) * ux + paf_value(a, f, my, yi, xi) * uy;
        sum = sum + s;                                                        // builtin sum(), left to right
        cnt += s > 0.05;
      }
      score_of(p, sum, cnt, nr);
    }
  }
  for (int i = tid; i < nA; i += 256) usedA[i] = 0;
  for (int j = tid; j < nB; j += 256) usedB[j] = 0;
  __syncthreads();
  // stable descending sort of the kept pairs (sorted(..., reverse=True)): rank = #(better)
  for (int p = tid; p < np; p += 256) {
    if (!pkeep[p]) continue;
    const double sp = pscore[p];
    int rank = 0;
    for (int q = 0; q < np; ++q)
      if (pkeep[q] && (pscore[q] > sp || (pscore[q] == sp && q < p))) ++rank;
    order[rank] = p;
    atomicAdd(&s_nkeep, 1);
  }
  __syncthreads();
  if (tid == 0) {
    double* cw = conns + (size_t)k * a.max_conns * 5;
    const int lim = nA < nB ? nA : nB;
    int m = 0;
    for (int r = 0; r < s_nkeep && m < lim; ++r) {
      const int p = order[r];
      const int i = p / nB, j = p - i * nB;
      if (usedA[i] || usedB[j]) continue;
      usedA[i] = usedB[j] = 1;
      if (m >= a.max_conns) { atomicExch(status, ISL_E_CAPACITY); break; }
      double* c = cw + (size_t)m * 5;
      c[0] = (double)(s_offA + i);
      c[1] = (double)(s_offB + j);
      c[2] = pscore[p];
      c[3] = (double)i;
      c[4] = (double)j;
      ++m;
    }
    n_conns[k] = m;
  }
}

// Person assembly (body.py:180-235), serial per frame: one lane per frame.
// Person assembly (body.py:164-232) -- one wave per frame.  The subset table
// lives in LDS when it fits (`in_lds`), so the row scans of the greedy merge are
// LDS ballots instead of dependent global loads; the kept rows are written to
// the record in one pass at the end.
constexpr int ASM_LDS_ROWS = 256;   // subset rows that fit the LDS table (256 x 27 doubles = 55 KB)
// The frame's connections and the candidate scores the merge adds are staged in LDS first, all
// lanes loading at once (ASM_CONN_CACHE of them; more: read in place): the serial merge then
// never waits on a global load (it waited on two per connection, ~75 us per 32-frame batch).
constexpr int ASM_CONN_CACHE = 512;   // x 5 doubles = 20 KB
// The merge with the table in registers: lane r holds subset row r, the limbs unrolled at compile
// time so that row[A] / row[B] are fixed registers.  The common connections -- one hit (a
// predicated update in the hit lane) or none (a new row) -- are then two compares and a ballot,
// with no LDS round trip on the chain.  The rare ones (two or three hits: the row merge and
// delete, the IndexError; a 65th row; the row cap) leave the register loop: the rows go to the
// table, the table merge takes that one connection (all the rest past 64 rows), and the rows come
// back.  Same operations in the same order as the table merge (body.py:186-226), so the same bits.
// (Unrolling the rare paths per limb too made a 200 KB kernel bound by instruction fetch.)
constexpr int kRegA25[24] = {1, 1, 2, 3, 1, 5, 6, 1, 8, 9, 10, 8, 12, 13, 0, 0, 15, 16, 11, 11, 14, 14, 22, 19};
constexpr int kRegB25[24] = {0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 24, 22, 21, 19, 23, 20};
constexpr int kRegACoco[19] = {1, 1, 2, 3, 5, 6, 1, 8, 9, 1, 11, 12, 1, 0, 14, 0, 15, 2, 5};
constexpr int kRegBCoco[19] = {2, 5, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 0, 14, 16, 15, 17, 16, 17};
constexpr int reg_limb_a(int model, int k) { return model == ISL_BODY25 ? kRegA25[k] : kRegACoco[k]; }
constexpr int reg_limb_b(int model, int k) { return model == ISL_BODY25 ? kRegB25[k] : kRegBCoco[k]; }

// limbs K .. NL-1 from connection (k_from, ci_from); returns 0 done, 2 stopped at (stop_k, stop_ci)
template <int MODEL, int RW, int NL, int K>
__device__ __forceinline__ int asm_reg_limbs(double (&v)[RW], int& rows, const double* s_conn, const int* s_koff,
                                             int lane, int max_rows, int k_from, int ci_from, int& stop_k,
                                             int& stop_ci) {
  if constexpr (K == NL) {
    return 0;
  } else {
    constexpr int A = reg_limb_a(MODEL, K), B = reg_limb_b(MODEL, K);
    constexpr bool NEW = MODEL == ISL_BODY25 ? true : K < 17;   // k < njoint - 2 (body.py:220)
    if (K >= k_from) {
      const int k0 = s_koff[K], m = s_koff[K + 1] - k0;
      for (int ci = K == k_from ? ci_from : 0; ci < m; ++ci) {
        const double* c = s_conn + (size_t)(k0 + ci) * 5;
        const double idA = c[0], idB = c[1];
        const bool hit = lane < rows && (v[A] == idA || v[B] == idB);
        const unsigned long long mask = __ballot(hit);
        const int found = __builtin_popcountll(mask);
        if (found >= 2 || (found == 0 && NEW && (rows >= 64 || rows >= max_rows))) {
          stop_k = K;
          stop_ci = ci;
          return 2;
        }
        if (found == 1) {
          if (lane == __builtin_ctzll(mask) && v[B] != idB) {
            v[B] = idB;
            v[RW - 1] = v[RW - 1] + 1.0;
            v[RW - 2] = v[RW - 2] + (c[4] + c[2]);
          }
        } else if constexpr (NEW) {
          if (lane == rows) {   // (lanes >= rows hold -1 everywhere: the caller keeps them so)
            v[A] = idA;
            v[B] = idB;
            v[RW - 1] = 2.0;
            v[RW - 2] = (c[3] + c[4]) + c[2];
          }
          ++rows;
        }
      }
    }
    return asm_reg_limbs<MODEL, RW, NL, K + 1>(v, rows, s_conn, s_koff, lane, max_rows, k_from, ci_from, stop_k,
                                                stop_ci);
  }
}

// IN_LDS: the subset table in LDS (a template parameter, so that its accesses are ds_* rather
// than flat instructions: a runtime choice of the table's address space made every access a
// flat load / store with global latency, ~1600 cycles per connection of the serial merge)
// MODEL: ISL_BODY25 / ISL_COCO (the register merge); use_reg = 0 the table merge only (A/B)
template <bool IN_LDS, int MODEL>
__global__ void __launch_bounds__(64) assemble_kernel(GroupArgs a, int conn_cap, int use_reg) {
  constexpr bool in_lds = IN_LDS;
  extern __shared__ double s_asm[];
  double* s_subset = s_asm;
  double* s_conn = s_asm + (in_lds ? (size_t)a.max_rows * (a.njoint + 1) : 0);   // [ASM_CONN_CACHE][5]
  __shared__ int s_off[32], s_koff[33];
  const int f = blockIdx.x, lane = threadIdx.x;
  char* rec = a.result + (size_t)f * a.lay.record_bytes;
  int* status = (int*)(rec + a.lay.status);
  const int* n_peaks = (const int*)(rec + a.lay.n_peaks);
  const int* n_conns = (const int*)(rec + a.lay.n_conns);
  int* n_rows = (int*)(rec + a.lay.n_rows);
  const double* peaks = (const double*)(rec + a.lay.peaks);
  const double* conns = (const double*)(rec + a.lay.conns);
  double* out = (double*)(rec + a.lay.subset);
  double* subset = IN_LDS ? s_subset : out;
  ASTAMP(0);
  if (*status != ISL_OK) return;
  const int RW = a.njoint + 1;   // subset row width
  {
    // candidate id offsets per part and connection offsets per limb: exclusive scans over lanes
    int np = lane < a.njoint - 1 ? n_peaks[lane] : 0;
    int nc = lane < a.nlimbs ? max(n_conns[lane], 0) : 0;
    int sp = np, sc = nc;
    for (int o = 1; o < 64; o <<= 1) {
      const int up = __shfl_up(sp, o), uc = __shfl_up(sc, o);
      if (lane >= o) {
        sp += up;
        sc += uc;
      }
    }
    if (lane < 32) s_off[lane] = sp - np;
    if (lane < 33) s_koff[lane] = sc - nc;
  }
  __syncthreads();
  ASTAMP(1);
  auto score_of = [&](int part, double id) {
    return peaks[((size_t)part * a.max_peaks + (int)(id - s_off[part])) * 3 + 2];   // candidate[id, 2]
  };
  const int total = s_koff[a.nlimbs];
  const bool cached = total <= conn_cap;
  if (cached) {
    for (int it = lane; it < total; it += 64) {
      int k = 0;
      while (s_koff[k + 1] <= it) ++k;
      const int A = a.model == ISL_BODY25 ? kLimbs25[k][0] : kLimbsCoco[k][0];
      const int B = a.model == ISL_BODY25 ? kLimbs25[k][1] : kLimbsCoco[k][1];
      const double* c = conns + ((size_t)k * a.max_conns + (it - s_koff[k])) * 5;
      const double idA = c[0], idB = c[1];
      double* e = s_conn + (size_t)it * 5;
      e[0] = idA;
      e[1] = idB;
      e[2] = c[2];
      e[3] = score_of(A, idA);
      e[4] = score_of(B, idB);
    }
    __syncthreads();
  }
  ASTAMP(2);
  int rows = 0;
  // the merge, instantiated per connection source (cache / record) so that every access is typed
  // (k_start, ci_start): the first connection; limit: how many to take (the register merge hands
  // over single connections)
  auto merge = [&](auto cache_tag, int k_start, int ci_start, int limit) -> bool {
  constexpr bool CACHED = decltype(cache_tag)::value;
  for (int k = k_start; k < a.nlimbs; ++k) {
    // (the staged counts: special_k's -1 is 0 there, and a limb without connections does nothing
    // either way -- no dependent global load per limb)
    const int m = s_koff[k + 1] - s_koff[k];
    if (m <= 0) continue;                // special_k
    const int A = a.model == ISL_BODY25 ? kLimbs25[k][0] : kLimbsCoco[k][0];
    const int B = a.model == ISL_BODY25 ? kLimbs25[k][1] : kLimbsCoco[k][1];
    const double* cw = conns + (size_t)k * a.max_conns * 5;
    for (int ci = k == k_start ? ci_start : 0; ci < m; ++ci) {
      if (limit-- == 0) return true;
      // (two typed branches, so that the cached reads are ds_* and not flat loads)
      double idA, idB, sc, sA = 0.0, sB = 0.0;
      if constexpr (CACHED) {
        const double* c = s_conn + (size_t)(s_koff[k] + ci) * 5;
        idA = c[0];
        idB = c[1];
        sc = c[2];
        sA = c[3];
        sB = c[4];
      } else {
        const double* c = cw + (size_t)ci * 5;
        idA = c[0];
        idB = c[1];
        sc = c[2];
      }
      // rows j with subset[j][A] == idA or subset[j][B] == idB, in order (body.py:191-196); the
      // scan also reads the first 64 rows' [B], count and score, which the one-row update takes
      // by lane exchange instead of dependent LDS reads
      int hit[2] = {-1, -1}, found = 0;
      double rb = 0.0, rcnt = 0.0, rsc = 0.0;
      for (int r0 = 0; r0 < rows; r0 += 64) {
        const int r = r0 + lane;
        bool hitr = false;
        if (r < rows) {
          const double* row = subset + (size_t)r * RW;
          const double ra = row[A], rbb = row[B];
          if (r0 == 0) {
            rb = rbb;
            rcnt = row[RW - 1];
            rsc = row[RW - 2];
          }
          hitr = ra == idA || rbb == idB;
        }
        unsigned long long mask = __ballot(hitr);
        while (mask && found < 3) {
          const int j = __builtin_ctzll(mask);
          mask &= mask - 1;
          if (found < 2) hit[found] = r0 + j;
          ++found;
        }
        if (found == 3) break;
      }
      if (found == 3) {                  // body.py:196 IndexError
        if (lane == 0) *status = ISL_E_INDEX;
        return false;
      }
      if (found == 1) {
        double* row = subset + (size_t)hit[0] * RW;
        if (hit[0] < 64) {
          // (a single wave: its LDS / global operations on the table are ordered, no barrier)
          const double ob = __shfl(rb, hit[0]), oc = __shfl(rcnt, hit[0]), os = __shfl(rsc, hit[0]);
          if (ob != idB && lane == 0) {
            row[B] = idB;
            row[RW - 1] = oc + 1.0;
            row[RW - 2] = os + ((CACHED ? sB : score_of(B, idB)) + sc);
          }
        } else {
          const bool upd = row[B] != idB;
          __syncthreads();
          if (upd && lane == 0) {
            row[B] = idB;
            row[RW - 1] += 1.0;
            row[RW - 2] += (CACHED ? sB : score_of(B, idB)) + sc;
          }
        }
      } else if (found == 2) {
        double* r1 = subset + (size_t)hit[0] * RW;
        double* r2 = subset + (size_t)hit[1] * RW;
        bool ov = false;
        for (int q = lane; q < RW - 2; q += 64) ov |= (r1[q] >= 0.0) && (r2[q] >= 0.0);
        const bool overlap = __ballot(ov) != 0ull;
        __syncthreads();
        if (!overlap) {
          for (int q = lane; q < RW - 2; q += 64) r1[q] += r2[q] + 1.0;
          if (lane == 0) {
            r1[RW - 2] += r2[RW - 2];
            r1[RW - 1] += r2[RW - 1];
            r1[RW - 2] += sc;
          }
          __syncthreads();
          // np.delete(subset, j2, 0): every element after row j2 moves up one row;
          // each wave step loads its 64 elements before storing them
          const int tail = (rows - 1 - hit[1]) * RW;
          double* d = subset + (size_t)hit[1] * RW;
          for (int i0 = 0; i0 < tail; i0 += 64) {
            const int i = i0 + lane;
            const double v = i < tail ? d[i + RW] : 0.0;
            __syncthreads();
            if (i < tail) d[i] = v;
            __syncthreads();
          }
          --rows;
        } else if (lane == 0) {
          r1[B] = idB;
          r1[RW - 1] += 1.0;
          r1[RW - 2] += (CACHED ? sB : score_of(B, idB)) + sc;
        }
      } else if (k < a.njoint - 2) {
        if (rows >= a.max_rows) {
          if (lane == 0) *status = ISL_E_CAPACITY;
          return false;
        }
        double* row = subset + (size_t)rows * RW;
        const double sAB = lane == 0 ? (CACHED ? sA + sB : score_of(A, idA) + score_of(B, idB)) + sc : 0.0;
        for (int q = lane; q < RW; q += 64) row[q] = -1.0;
        __syncthreads();
        if (lane == 0) {
          row[A] = idA;
          row[B] = idB;
          row[RW - 1] = 2.0;
          row[RW - 2] = sAB;
        }
        ++rows;
      }
      // (the LDS table: one wave's LDS operations execute in order, so the next connection's
      // scan sees these writes without a barrier; the global table keeps it)
      if (!in_lds) __syncthreads();
    }
  }
  return true;
  };
  if (cached && use_reg) {
    constexpr int RWC = MODEL == ISL_BODY25 ? 27 : 20, NLC = MODEL == ISL_BODY25 ? 24 : 19;
    if (RW != RWC || a.nlimbs != NLC) {
      if (lane == 0) *status = ISL_E_ARG;
      return;
    }
    double v[RWC];
#pragma unroll
    for (int q = 0; q < RWC; ++q) v[q] = -1.0;
    int k_from = 0, ci_from = 0;
    while (true) {
      int stop_k = 0, stop_ci = 0;
      const int rc = asm_reg_limbs<MODEL, RWC, NLC, 0>(v, rows, s_conn, s_koff, lane, a.max_rows, k_from, ci_from,
                                                        stop_k, stop_ci);
      // the rows to the table (the prune below and the table merge read them there)
      if (lane < rows) {
#pragma unroll
        for (int q = 0; q < RWC; ++q) subset[(size_t)lane * RWC + q] = v[q];
      }
      __syncthreads();
      if (rc == 0) break;
      // the stopping connection on the table merge; past 64 rows (or at the cap) all the rest
      const bool rest = rows >= 64 || rows >= a.max_rows;
      if (!merge(std::true_type{}, stop_k, stop_ci, rest ? 0x7fffffff : 1)) return;
      if (rest) break;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < RWC; ++q) v[q] = lane < rows ? subset[(size_t)lane * RWC + q] : -1.0;
      k_from = stop_k;
      ci_from = stop_ci + 1;
    }
  } else if (!(cached ? merge(std::true_type{}, 0, 0, 0x7fffffff) : merge(std::false_type{}, 0, 0, 0x7fffffff))) {
    return;
  }
  ASTAMP(3);
  // prune (body.py:227-231): keep rows with count >= 4 and mean score >= 0.4, in order
  int w = 0;
  for (int r0 = 0; r0 < rows; r0 += 64) {
    const int r = r0 + lane;
    bool keep = false;
    if (r < rows) {
      const double* row = subset + (size_t)r * RW;
      keep = !(row[RW - 1] < 4.0 || row[RW - 2] / row[RW - 1] < 0.4);
    }
    const unsigned long long km = __ballot(keep);
    if (in_lds) {
      if (keep) {
        const int dst = w + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)km, 0u));
        for (int q = 0; q < RW; ++q) out[(size_t)dst * RW + q] = subset[(size_t)r * RW + q];
      }
    } else {
      // in place, in order (destination rows never pass their source rows)
      unsigned long long mm = km;
      int dst = w;
      while (mm) {
        const int j = __builtin_ctzll(mm);
        mm &= mm - 1;
        if (dst != r0 + j)
          for (int q = lane; q < RW; q += 64) out[(size_t)dst * RW + q] = out[(size_t)(r0 + j) * RW + q];
        ++dst;
        __syncthreads();
      }
    }
    w += __builtin_popcountll(km);
  }
  if (lane == 0) *n_rows = w;
  ASTAMP(4);
}

// ---------------------------------------------------------------------------
// Hand peaks (hand.py:58-73): 8-connected components of the thresholded blur,
// the component with the largest np.sum(map_ori[label == i]) (first on ties,
// labels numbered in raster order of their first pixel), then util.npmax of
// map_ori with every other pixel zeroed.  One workgroup per (crop, part).
// ---------------------------------------------------------------------------

// parent arrays live in LDS (planes up to CC_LDS_MAX pixels: workgroup-scope
// atomics, ds_* instructions) or in global scratch (agent scope)
typedef __attribute__((address_space(3))) int lds_int;
template <typename PT> struct UfScope { static constexpr int v = __HIP_MEMORY_SCOPE_AGENT; };
template <> struct UfScope<lds_int*> { static constexpr int v = __HIP_MEMORY_SCOPE_WORKGROUP; };

template <typename PT>
__device__ __forceinline__ int ld_parent(PT p, int x) {
  return __hip_atomic_load(p + x, __ATOMIC_RELAXED, UfScope<PT>::v);
}

// find with path halving: a non-root's parent is only ever replaced by one of its
// ancestors (halving stores here; the union CAS only touches roots), so the
// relaxed stores are race-safe and chains stay short.  Without it a plane that
// is one big component (random weights) built O(P)-long chains: 7 ms per crop.
template <typename PT>
__device__ int uf_find(PT parent, int x) {
  while (true) {
    const int p = ld_parent(parent, x);
    if (p == x) return x;
    const int gp = ld_parent(parent, p);
    if (gp == p) return p;
    __hip_atomic_store(parent + x, gp, __ATOMIC_RELAXED, UfScope<PT>::v);
    x = gp;
  }
}

// read-only walk to the root, for the final labelling pass: each pixel's owner then
// stores the root, and nobody else writes that slot, so every parent ends as its
// root.  (A halving find here could, racing with the owner, overwrite a stored
// root with a mere ancestor.)
template <typename PT>
__device__ int uf_root(PT parent, int x) {
  while (true) {
    const int p = ld_parent(parent, x);
    if (p == x) return x;
    x = p;
  }
}

// lock-free union: hook the larger root under the smaller with a CAS, so the
// final root of every component is its smallest raster index (= label order).
template <typename PT>
__device__ void uf_union(PT parent, int a, int b) {
  while (true) {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    if (a == b) return;
    if (a < b) { const int t = a; a = b; b = t; }
    int expected = a;
    if (__hip_atomic_compare_exchange_strong(parent + a, &expected, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             UfScope<PT>::v))
      return;
  }
}

// numpy pairwise_sum (loops_utils.h.src): < 8 sequential from 0; <= 128: 8
// accumulators; else split at n/2 rounded down to a multiple of 8.
__device__ double np_pairwise(const double* a, int n) {
  // iterative post-order walk of the split tree (depth <= 32)
  struct Frame { int off, len, state; double left; };
  Frame st[32];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Frame& f = st[sp];
    if (f.len <= 128) {
      double res;
      const double* x = a + f.off;
      if (f.len < 8) {
        res = 0.0;
        for (int i = 0; i < f.len; ++i) res += x[i];
      } else {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = x[k];
        int i = 8;
        for (; i < f.len - (f.len % 8); i += 8)
          for (int k = 0; k < 8; ++k) r[k] += x[i + k];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < f.len; ++i) res += x[i];
      }
      ret = res;
      --sp;
      continue;
    }
    int n2 = f.len / 2;
    n2 -= n2 % 8;
    if (f.state == 0) {
      f.state = 1;
      st[++sp] = {f.off, n2, 0, 0.0};
    } else if (f.state == 1) {
      f.left = ret;
      f.state = 2;
      st[++sp] = {f.off + n2, f.len - n2, 0, 0.0};
    } else {
      ret = f.left + ret;
      --sp;
    }
  }
  return ret;
}

// numpy's leaf: < 8 sequential from 0; <= 128: 8 accumulators, then the tail
__device__ __forceinline__ double np_leaf(const double* x, int len) {
  if (len < 8) {
    double res = 0.0;
    for (int i = 0; i < len; ++i) res += x[i];
    return res;
  }
  double r[8];
  for (int k = 0; k < 8; ++k) r[k] = x[k];
  int i = 8;
  for (; i < len - (len % 8); i += 8)
    for (int k = 0; k < 8; ++k) r[k] += x[i + k];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < len; ++i) res += x[i];
  return res;
}

// Block-cooperative np.sum with numpy's exact association (same result as np_sum).
// A full 8192-element buffer always has the same tree -- 64 leaves of 128 elements,
// paired level by level (n2 = n/2 is a multiple of 8 down to 128) -- so one wave
// sums a buffer: a leaf per lane, then 6 shuffle levels, every wave on its own
// buffer.  The partial last buffer takes the general path: thread 0 lists the
// leaves of its split tree, the block sums them, thread 0 combines them in tree
// order.  Buffers are added left to right.  Every thread of the block must call it;
// the result is returned to all of them.
// numpy's pairwise sum of one full 8192-element buffer by one wave (the sum in lane 0)
__device__ __forceinline__ double np_buf8192_wave(const double* buf) {
  const int lane = threadIdx.x & 63;
      // the 64 leaves of 128, eight at a time: lane j of a group of 8 keeps np_leaf's
      // accumulator r[j] (coalesced 64-byte rows instead of a 1 KiB-strided leaf per
      // lane), then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) as xor butterflies (a + b ==
      // b + a exactly); leaf 8k+g ends in lane 8k+g
      const int g8 = lane >> 3, j8 = lane & 7;
      double v = 0.0;
      for (int k = 0; k < 8; ++k) {
        const double* leaf = buf + (k * 8 + g8) * 128 + j8;
        double r = leaf[0];
#pragma unroll
        for (int i = 8; i < 128; i += 8) r += leaf[i];
        r += __shfl_xor(r, 1, 64);
        r += __shfl_xor(r, 2, 64);
        r += __shfl_xor(r, 4, 64);
        const double t = __shfl(r, (lane & 7) * 8, 64);   // group (lane & 7) holds leaf 8k + (lane & 7)
        if (g8 == k) v = t;
      }
#pragma unroll
      for (int half = 32; half >= 1; half >>= 1) {
        const double x0 = __shfl(v, 2 * lane, 64), x1 = __shfl(v, 2 * lane + 1, 64);
        if (lane < half) v = x0 + x1;
      }
  return v;
}

// np_sum_block with the full buffers' sums already computed (pre[b], cc_bufsum_kernel)
// when pre != nullptr
__device__ double np_sum_block(const double* a, int n, const double* pre = nullptr) {
  constexpr int MAXL = 128;   // leaves of a < 8192-element tree have 65..128 elements
  __shared__ int s_loff[MAXL], s_llen[MAXL], s_nl;
  __shared__ double s_lsum[MAXL];
  __shared__ double s_part[32];
  __shared__ double s_tot;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int nfull = n / 8192;
  if (pre) {
    if (tid == 0)
      for (int b = 0; b < nfull; ++b) s_tot = b == 0 ? pre[0] : s_tot + pre[b];
    __syncthreads();
  }
  for (int g = 0; !pre && g < nfull; g += nw) {
    const int b = g + wave;
    if (b < nfull) {
      const double v = np_buf8192_wave(a + (size_t)b * 8192);
      if (lane == 0) s_part[wave] = v;
    }
    __syncthreads();
    if (tid == 0)
      for (int k = 0; k < nw && g + k < nfull; ++k) s_tot = g + k == 0 ? s_part[k] : s_tot + s_part[k];
    __syncthreads();
  }
  const int i0 = nfull * 8192, len0 = n - i0;
  if (len0 > 0) {
    if (tid == 0) {   // pre-order leaf list
      int st_off[32], st_len[32], sp = 0, nl = 0;
      st_off[0] = i0; st_len[0] = len0;
      while (sp >= 0) {
        const int off = st_off[sp], len = st_len[sp];
        --sp;
        if (len <= 128) { s_loff[nl] = off; s_llen[nl] = len; ++nl; continue; }
        int n2 = len / 2;
        n2 -= n2 % 8;
        ++sp; st_off[sp] = off + n2; st_len[sp] = len - n2;   // right pushed first: left pops first
        ++sp; st_off[sp] = off; st_len[sp] = n2;
      }
      s_nl = nl;
    }
    __syncthreads();
    for (int l = tid; l < s_nl; l += blockDim.x) s_lsum[l] = np_leaf(a + s_loff[l], s_llen[l]);
    __syncthreads();
    if (tid == 0) {   // post-order combination (left + right at every split)
      struct F { int len, state; double left; };
      F st[32];
      int sp = 0, leaf = 0;
      st[0] = {len0, 0, 0.0};
      double ret = 0.0;
      while (sp >= 0) {
        F& f = st[sp];
        if (f.len <= 128) { ret = s_lsum[leaf++]; --sp; continue; }
        int n2 = f.len / 2;
        n2 -= n2 % 8;
        if (f.state == 0) { f.state = 1; st[++sp] = {n2, 0, 0.0}; }
        else if (f.state == 1) { f.left = ret; f.state = 2; st[++sp] = {f.len - n2, 0, 0.0}; }
        else { ret = f.left + ret; --sp; }
      }
      s_tot = nfull == 0 ? ret : s_tot + ret;
    }
    __syncthreads();
  }
  const double r = s_tot;
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(1024) np_sum_debug_kernel(const double* a, int n, double* out) {
  const double s = np_sum_block(a, n);
  if (threadIdx.x == 0) out[0] = s;
}

// np.sum of a contiguous float64 array: pairwise sums of 8192-element buffers, added left to right
__device__ double np_sum(const double* a, int n) {
  double s = 0.0;
  for (int i = 0; i < n; i += 8192) {
    const double p = np_pairwise(a + i, min(8192, n - i));
    s = i == 0 ? p : s + p;
  }
  return s;
}

constexpr int CC_LDS_MAX = 36864;   // plane pixels whose parent array fits LDS (144 KB)
constexpr int CC_CHUNK = 4096;      // pixels per row chunk of the large-plane path
constexpr int CC_WMAX = 8192;       // widest plane the large-plane path takes (LDS chunk parents)
constexpr int CC_MAXC = 64;         // candidate components kept per plane

// per-plane results of the large-plane pre-pass
struct CcStats {
  int count;                        // foreground pixels
  int ncand;                        // components whose approximate sum reaches the candidate bar
  unsigned long long maxbits;       // largest approximate component sum (bits of a positive double)
  int cand[CC_MAXC];                // their roots, unordered
};

// Adds map[p] into vals[root of p] for p in [p0, p1): runs of equal roots are summed
// in a register and flushed with one atomic; the last flush of a wave whose lanes all
// hold the same root (a plane that is one big component: random weights) is summed
// across the wave first.  Order-free (see the candidate pass).
template <typename PT>
__device__ __forceinline__ void cc_root_sums(PT parent, const double* map, double* vals, int p0, int p1) {
  int cur = -1;
  double acc = 0.0;
  for (int p = p0; p < p1; ++p) {
    const int r = parent[p];
    if (r < 0) continue;
    if (r != cur) {
      if (cur >= 0) atomicAdd(&vals[cur], acc);
      cur = r;
      acc = 0.0;
    }
    acc += map[p];
  }
  const unsigned long long act = __ballot(cur >= 0);      // lanes without foreground: no vote
  const int r0 = act ? __shfl(cur, __builtin_ctzll(act), 64) : -1;
  if (act && __all(cur < 0 || cur == r0)) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&vals[r0], acc);
  } else if (cur >= 0) {
    atomicAdd(&vals[cur], acc);
  }
}

// Large-plane path (planes above CC_LDS_MAX: hand crops of HD frames reach 600 x 600
// px), a sequence of multi-block launches over (plane, row chunk of <= CC_CHUNK px):
//   cc_local  -- connected components of the chunk in LDS (the lock-free union-find at
//                workgroup scope), labels written as global pixel indices;
//   cc_merge  -- unions across chunk boundaries only (the chunk's first row with the
//                row above), on the global parents: a few hundred global CAS per
//                chunk instead of ~4 per pixel with dependent L2 round trips;
//   cc_find   -- every parent becomes its root (smallest raster index of the component);
//   cc_sum    -- approximate root sums and the foreground count;
//   cc_stats  -- the largest approximate sum, then cc_cand the candidate roots;
//   hand_cc_kernel<false, true> -- exact sums of the candidates and the argmax.
__global__ void __launch_bounds__(256) cc_local_kernel(const unsigned long long* __restrict__ mask, int h, int w,
                                                       int words, int rows, int chunks, int* __restrict__ parent_all,
                                                       double* __restrict__ vals_all, CcStats* __restrict__ stats) {
  __shared__ int s_lp[CC_WMAX > CC_CHUNK ? CC_WMAX : CC_CHUNK];
  // the chunk's mask rows in LDS (unions stay inside the chunk); chunks of very narrow
  // planes (many rows of one word) read the global mask instead
  constexpr int MW = 256;
  __shared__ unsigned long long s_mk[MW];
  lds_int* lp = (lds_int*)s_lp;
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int y0 = c * rows, y1 = min(h, y0 + rows), base = y0 * w, n = (y1 - y0) * w;
  const unsigned long long* mk = mask + (size_t)plane * h * words + (size_t)y0 * words;
  int* parent = parent_all + (size_t)plane * h * w;
  if (c == 0 && threadIdx.x == 0) { stats[plane].count = 0; stats[plane].ncand = 0; stats[plane].maxbits = 0; }
  const int nw = (y1 - y0) * words;
  const bool in_lds = nw <= MW;
  if (in_lds)
    for (int i = threadIdx.x; i < nw; i += 256) s_mk[i] = mk[i];
  __syncthreads();
  auto bit = [&](int yl, int x) -> bool {
    const int q = yl * words + (x >> 6);
    return ((in_lds ? s_mk[q] : mk[q]) >> (x & 63)) & 1ull;
  };
  auto word = [&](int yl, int k) -> unsigned long long {
    const int q = yl * words + k;
    return in_lds ? s_mk[q] : mk[q];
  };
  // horizontal runs without atomics: every foreground pixel's parent is the first pixel
  // of its run (the highest clear mask bit below it, across words)
  for (int i = threadIdx.x; i < n; i += 256) {
    const int yl = i / w, x = i - yl * w;
    if (!bit(yl, x)) { lp[i] = -1; continue; }
    int k = x >> 6;
    unsigned long long z = ~word(yl, k) & ((1ull << (x & 63)) - 1ull);   // clear bits below x
    while (!z && k > 0) z = ~word(yl, --k);
    const int xs = z ? (k << 6) + 64 - __clzll((long long)z) : 0;
    lp[i] = yl * w + xs;
  }
  __syncthreads();
  // vertical: one union per 8-adjacent (run, run above) pair, as cc_merge_kernel (a pixel
  // unions with an upper neighbour when either starts its run)
  for (int i = threadIdx.x; i < n; i += 256) {
    const int yl = i / w, x = i - yl * w;
    if (yl == 0 || lp[i] < 0) continue;
    const bool start = lp[i] == i;
#pragma unroll
    for (int d = -1; d <= 1; ++d) {
      const int xu = x + d;
      if (xu < 0 || xu >= w || !bit(yl - 1, xu)) continue;
      if (start || xu == 0 || !bit(yl - 1, xu - 1)) uf_union(lp, i, i - w + d);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256)
    if (ld_parent(lp, i) >= 0) __hip_atomic_store(lp + i, uf_root(lp, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) parent[base + i] = lp[i] >= 0 ? base + lp[i] : -1;
  (void)vals_all;   // the root accumulators are zeroed by cc_find_kernel (roots only)
}

__global__ void __launch_bounds__(256) cc_merge_kernel(const unsigned long long* __restrict__ mask, int h, int w,
                                                       int words, int rows, int chunks, int* __restrict__ parent_all) {
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  if (c == 0) return;
  const int y = c * rows;
  const unsigned long long* mk = mask + (size_t)plane * h * words;
  int* parent = parent_all + (size_t)plane * h * w;
  auto bit = [&](int yy, int x) -> bool { return (mk[(size_t)yy * words + (x >> 6)] >> (x & 63)) & 1ull; };
  // Runs of foreground pixels along a row are one local component each, so one union
  // per 8-adjacent (run below, run above) pair suffices: pixel x unions with an upper
  // neighbour x' when x' starts its run or x starts its own.  Every adjacent pair of
  // runs meets one of the two cases (the upper run starts inside [x0-1, x1+1] of the
  // lower run [x0, x1], or covers x0-1), and a dense plane makes ~3 unions per boundary
  // instead of ~3 per pixel, all on the same two roots.
  for (int x = threadIdx.x; x < w; x += 256) {
    if (!bit(y, x)) continue;
    const int p = y * w + x;
    const bool start = x == 0 || !bit(y, x - 1);
#pragma unroll
    for (int d = -1; d <= 1; ++d) {
      const int xu = x + d;
      if (xu < 0 || xu >= w || !bit(y - 1, xu)) continue;
      if (start || xu == 0 || !bit(y - 1, xu - 1)) uf_union(parent, p, p - w + d);
    }
  }
}

// labelling: every pixel's parent becomes its root (roots are final once every union
// is done; uf_root)
__global__ void __launch_bounds__(256) cc_find_kernel(int h, int w, int rows, int chunks, int* __restrict__ parent_all,
                                                      double* __restrict__ vals_all) {
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  int* parent = parent_all + (size_t)plane * P;
  double* vals = vals_all + (size_t)plane * P;
  // a thread's pixels (256 apart) mostly share their chunk-local root: its walk up the
  // merged chunk roots is done once and reused while that local root repeats (roots are
  // final here; p's own slot is written only by this thread)
  int last_q = -1, last_r = -1;
  for (int p = p0 + threadIdx.x; p < p1; p += 256) {
    const int q = ld_parent(parent, p);
    if (q < 0) continue;
    int r;
    if (q == last_q) {
      r = last_r;
    } else {
      r = uf_root(parent, q);
      last_q = q;
      last_r = r;
    }
    __hip_atomic_store(parent + p, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r == p) vals[p] = 0.0;   // a root: its cc_sum accumulator (only roots are ever read)
  }
}

// Per-block table of component sums (root -> partial sum) in LDS: a thread's run of equal
// roots is flushed into the table, and the table into the roots' global sums once per block.
// Flushing runs straight to global memory (round 5) made the random-weight hand maps -- large
// components interleaved along a thread's 256-pixel stride -- thousands of fp64 atomics on
// the same few addresses per plane: 625 us of the 1.7 ms post of a 1080 px crop
// (profiles/r06/fr6/post_trace).  The sums only pick the candidate components (within a
// relative 1e-9 of the largest, cc_cand_kernel); the winners' exact numpy sums come from
// cc_scatter / cc_bufsum, so the order of these additions does not reach a result.
constexpr int CC_HASH = 1024;   // table slots per block (4096 pixels per chunk at most)
constexpr int CC_PROBE = 8;     // linear probes before a run goes straight to its root
__global__ void __launch_bounds__(256) cc_sum_kernel(const double* __restrict__ planes, int h, int w, int rows,
                                                     int chunks, const int* __restrict__ parent_all,
                                                     double* __restrict__ vals_all, CcStats* __restrict__ stats) {
  __shared__ int s_key[CC_HASH];
  __shared__ double s_val[CC_HASH];
  __shared__ int s_cnt;
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  const int* parent = parent_all + (size_t)plane * P;
  const double* map = planes + (size_t)plane * P;
  double* vals = vals_all + (size_t)plane * P;
  for (int i = threadIdx.x; i < CC_HASH; i += 256) {
    s_key[i] = -1;
    s_val[i] = 0.0;
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  auto flush = [&](int r, double a) {
    const unsigned hsh = ((unsigned)r * 2654435761u) >> 22;   // 10 bits (CC_HASH)
#pragma unroll 1
    for (int q = 0; q < CC_PROBE; ++q) {
      const int slot = (int)((hsh + q) & (CC_HASH - 1));
      const int old = atomicCAS(&s_key[slot], -1, r);
      if (old == -1 || old == r) {
        atomicAdd(&s_val[slot], a);
        return;
      }
    }
    atomicAdd(&vals[r], a);   // a crowded table: this run goes to its root directly
  };
  // Block-strided pixels: every load is one coalesced row segment (a contiguous run per
  // thread made each load touch 64 cache lines); a chunk is <= CC_CHUNK = 16 x 256 pixels:
  // every parent load of the thread, then every value load, in flight together
  constexpr int PER = CC_CHUNK / 256;
  int cnt = 0, cur = -1;
  double acc = 0.0;
  for (int q0 = p0; q0 < p1; q0 += CC_CHUNK) {
    int r[PER];
    double v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int p = q0 + threadIdx.x + 256 * k;
      r[k] = p < p1 ? parent[p] : -1;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = r[k] >= 0 ? map[q0 + threadIdx.x + 256 * k] : 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (r[k] < 0) continue;
      ++cnt;
      if (r[k] != cur) {
        if (cur >= 0) flush(cur, acc);
        cur = r[k];
        acc = 0.0;
      }
      acc += v[k];
    }
  }
  if (cur >= 0) flush(cur, acc);
  if (cnt) atomicAdd(&s_cnt, cnt);
  __syncthreads();
  for (int i = threadIdx.x; i < CC_HASH; i += 256)
    if (s_key[i] >= 0) atomicAdd(&vals[s_key[i]], s_val[i]);
  if (threadIdx.x == 0 && s_cnt) atomicAdd(&stats[plane].count, s_cnt);
}

__global__ void __launch_bounds__(256) cc_stats_kernel(int h, int w, int rows, int chunks,
                                                       const int* __restrict__ parent_all,
                                                       const double* __restrict__ vals_all, CcStats* __restrict__ stats) {
  __shared__ double s_m[4];
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  const int* parent = parent_all + (size_t)plane * P;
  const double* vals = vals_all + (size_t)plane * P;
  double m = 0.0;                                           // sums are of values > thre > 0
  for (int p = p0 + threadIdx.x; p < p1; p += 256)
    if (parent[p] == p) m = fmax(m, vals[p]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmax(fmax(s_m[0], s_m[1]), fmax(s_m[2], s_m[3]));
    if (m > 0.0) atomicMax(&stats[plane].maxbits, (unsigned long long)__double_as_longlong(m));
  }
}

__global__ void __launch_bounds__(256) cc_cand_kernel(int h, int w, int rows, int chunks,
                                                      const int* __restrict__ parent_all,
                                                      const double* __restrict__ vals_all, CcStats* __restrict__ stats) {
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  const int* parent = parent_all + (size_t)plane * P;
  const double* vals = vals_all + (size_t)plane * P;
  CcStats& st = stats[plane];
  if (st.count == 0) return;
  const double thr_c = __longlong_as_double((long long)st.maxbits) * (1.0 - 1e-9);
  for (int p = p0 + threadIdx.x; p < p1; p += 256)
    if (parent[p] == p && vals[p] >= thr_c) {
      const int slot = atomicAdd(&st.ncand, 1);
      if (slot < CC_MAXC) st.cand[slot] = p;
    }
}

// Fast finish for planes with at most CC_KFAST candidate components (in practice one):
// per (plane, chunk) the candidates' pixel counts and first maxima (cc_count), then
// their values compacted in raster order into `vals` (cc_scatter, each chunk at the
// prefix of the counts before it), so the per-plane kernel only runs numpy's
// pairwise sums and reduces the chunk maxima.
constexpr int CC_KFAST = 4;
struct CcChunk {
  int count[CC_KFAST];
  int besti[CC_KFAST];
  double bestv[CC_KFAST];
};

__device__ __forceinline__ void cc_pick2(double& v, int& i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__global__ void __launch_bounds__(256) cc_count_kernel(const double* __restrict__ planes, int h, int w, int rows,
                                                       int chunks, const int* __restrict__ parent_all,
                                                       const CcStats* __restrict__ stats, CcChunk* __restrict__ ck) {
  __shared__ int s_c[4];
  __shared__ double s_v[4];
  __shared__ int s_i[4];
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int nk = stats[plane].ncand;
  if (stats[plane].count == 0 || nk < 1 || nk > CC_KFAST) return;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  const int* parent = parent_all + (size_t)plane * P;
  const double* map = planes + (size_t)plane * P;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  CcChunk& out = ck[(size_t)plane * chunks + c];
  for (int k = 0; k < nk; ++k) {
    const int root = stats[plane].cand[k];
    int cnt = 0, bi = 0x7fffffff;
    double bv = -1.0;
    for (int p = p0 + threadIdx.x; p < p1; p += 256)
      if (parent[p] == root) {
        ++cnt;
        cc_pick2(bv, bi, map[p], p);
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cnt += __shfl_xor(cnt, o, 64);
      cc_pick2(bv, bi, __shfl_xor(bv, o, 64), __shfl_xor(bi, o, 64));
    }
    if (lane == 0) { s_c[wave] = cnt; s_v[wave] = bv; s_i[wave] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      double v = -1.0;
      int i = 0x7fffffff;
      for (int q = 0; q < 4; ++q) { t += s_c[q]; cc_pick2(v, i, s_v[q], s_i[q]); }
      out.count[k] = t; out.bestv[k] = v; out.besti[k] = i;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) cc_scatter_kernel(const double* __restrict__ planes, int h, int w, int rows,
                                                         int chunks, const int* __restrict__ parent_all,
                                                         const CcStats* __restrict__ stats,
                                                         const CcChunk* __restrict__ ck, double* __restrict__ vals_all) {
  __shared__ int s_w[4], s_base;
  const int plane = blockIdx.x / chunks, c = blockIdx.x % chunks;
  const int nk = stats[plane].ncand;
  if (stats[plane].count == 0 || nk < 1 || nk > CC_KFAST) return;
  const int P = h * w, p0 = c * rows * w, p1 = min(P, p0 + rows * w);
  const int* parent = parent_all + (size_t)plane * P;
  const double* map = planes + (size_t)plane * P;
  double* vals = vals_all + (size_t)plane * P;
  const CcChunk* pc = ck + (size_t)plane * chunks;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < nk; ++k) {
    const int root = stats[plane].cand[k];
    if (threadIdx.x == 0) {   // region of candidate k, then this chunk's place in it
      int base = 0;
      for (int q = 0; q < k; ++q)
        for (int cc = 0; cc < chunks; ++cc) base += pc[cc].count[q];
      for (int cc = 0; cc < c; ++cc) base += pc[cc].count[k];
      s_base = base;
    }
    __syncthreads();
    int o = s_base;
    // raster order, 256-pixel segments: each thread one pixel per segment (coalesced),
    // its slot = the segment's base + the members before it (ballot prefix per wave,
    // wave totals through LDS)
    for (int s0 = p0; s0 < p1; s0 += 256) {
      const int p = s0 + threadIdx.x;
      const bool in = p < p1 && parent[p] == root;
      const unsigned long long bal = __ballot(in);
      if (lane == 0) s_w[wave] = __popcll(bal);
      __syncthreads();
      int before = o;
      for (int q = 0; q < wave; ++q) before += s_w[q];
      if (in) vals[before + __popcll(bal & ((1ull << lane) - 1ull))] = map[p];
      o += s_w[0] + s_w[1] + s_w[2] + s_w[3];
      __syncthreads();
    }
  }
}

constexpr int CC_NT = 1024;   // threads per plane (one workgroup per (crop, part))
constexpr int CC_NW = CC_NT / 64;
constexpr int CC_RUN = 8;     // consecutive pixels per thread and round of the per-plane passes

__device__ __forceinline__ double cc_block_max(double v, double* s_d) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s_d[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = s_d[0];
#pragma unroll
  for (int k = 1; k < CC_NW; ++k) r = fmax(r, s_d[k]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ int cc_block_sum(int v, int* s_i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_i[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int k = 0; k < CC_NW; ++k) r += s_i[k];
  __syncthreads();
  return r;
}

__device__ __forceinline__ int cc_block_min(int v, int* s_i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) s_i[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = s_i[0];
#pragma unroll
  for (int k = 1; k < CC_NW; ++k) r = min(r, s_i[k]);
  __syncthreads();
  return r;
}

// (value, index) with the larger value, the smaller index on ties (first max)
__device__ __forceinline__ void cc_pick(double& v, int& i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__device__ __forceinline__ int cc_block_argmax(double v, int i, double* s_d, int* s_i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cc_pick(v, i, __shfl_xor(v, o, 64), __shfl_xor(i, o, 64));
  if ((threadIdx.x & 63) == 0) { s_d[threadIdx.x >> 6] = v; s_i[threadIdx.x >> 6] = i; }
  __syncthreads();
  double bv = s_d[0];
  int bi = s_i[0];
#pragma unroll
  for (int k = 1; k < CC_NW; ++k) cc_pick(bv, bi, s_d[k], s_i[k]);
  __syncthreads();
  return bi;
}

// inclusive prefix sum of v over the CC_NT-thread block; total = the block's sum
__device__ __forceinline__ int cc_block_scan(int v, int* s_i, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  if (lane == 63) s_i[wave] = v;
  __syncthreads();
  int off = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < CC_NW; ++k) {
    const int t = s_i[k];
    off += k < wave ? t : 0;
    total += t;
  }
  __syncthreads();
  return v + off;
}

// LDSP: parents in LDS (planes up to CC_LDS_MAX px).  PRE: parents (roots) and root
// sums come from the multi-block pre-pass (global parents).  The per-plane passes
// walk CC_RUN consecutive pixels per thread and round with 1024 threads: a plane of a
// 600 px crop is ~44 rounds per pass, not the ~1400 dependent rounds of a
// 256-thread, one-pixel-per-round loop.
// The full 8192-element buffers of every candidate's compacted values (cc_scatter) summed
// across many blocks, one wave per buffer (numpy's exact tree); hand_cc_kernel<false, true>
// adds them left to right.  bsum[(plane * CC_KFAST + k) * maxb + b].
__global__ void __launch_bounds__(256) cc_bufsum_kernel(const CcStats* __restrict__ stats,
                                                        const CcChunk* __restrict__ ck, int chunks, int P,
                                                        const double* __restrict__ vals_all, double* __restrict__ bsum,
                                                        int maxb) {
  __shared__ int s_tot[CC_KFAST];
  const int plane = blockIdx.x, nk = stats[plane].ncand;
  if (stats[plane].count == 0 || nk < 1 || nk > CC_KFAST) return;
  const CcChunk* pc = ck + (size_t)plane * chunks;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < CC_KFAST) s_tot[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < nk; ++k) {
    int t = 0;
    for (int c = threadIdx.x; c < chunks; c += 256) t += pc[c].count[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) atomicAdd(&s_tot[k], t);
  }
  __syncthreads();
  const double* vals = vals_all + (size_t)plane * P;
  for (int k = 0, base = 0; k < nk; base += s_tot[k], ++k) {
    const int nb = s_tot[k] / 8192;
    for (int b = blockIdx.y * 4 + wave; b < nb; b += gridDim.y * 4) {
      const double v = np_buf8192_wave(vals + base + (size_t)b * 8192);
      if (lane == 0) bsum[((size_t)plane * CC_KFAST + k) * maxb + b] = v;
    }
  }
}

template <bool LDSP, bool PRE>
__global__ void __launch_bounds__(CC_NT) hand_cc_kernel(const double* __restrict__ planes,
                                                        const unsigned long long* __restrict__ mask, int h, int w,
                                                        int words, int* __restrict__ parent_all,
                                                        double* __restrict__ vals_all, const CcStats* __restrict__ stats,
                                                        const CcChunk* __restrict__ ck, int chunks,
                                                        long long* __restrict__ out,
                                                        const double* __restrict__ bsum_all, int maxb) {
  extern __shared__ int s_dyn[];
  const int plane = blockIdx.x;   // crop * 21 + part
  const int P = h * w, tid = threadIdx.x;
  const double* map = planes + (size_t)plane * P;
  const unsigned long long* mk = mask + (size_t)plane * h * words;
  typedef typename std::conditional<LDSP, lds_int*, int*>::type PT;
  PT parent;
  if constexpr (LDSP) parent = (lds_int*)s_dyn;
  else parent = parent_all + (size_t)plane * P;
  double* vals = vals_all + (size_t)plane * P;
  auto bit = [&](int y, int x) -> bool { return (mk[(size_t)y * words + (x >> 6)] >> (x & 63)) & 1ull; };
  __shared__ int s_i[CC_NW];
  __shared__ double s_d[CC_NW];
  constexpr int MAXC = CC_MAXC;
  __shared__ int s_cand[MAXC];
  __shared__ int s_ncand;
  __shared__ double s_best_sum;
  __shared__ int s_best_root;
  int local = 0;
  if constexpr (PRE) {
    local = tid == 0 ? stats[plane].count : 0;
  } else {
    for (int q = tid * CC_RUN; q < P; q += CC_NT * CC_RUN) {
#pragma unroll
      for (int k = 0; k < CC_RUN; ++k) {
        const int p = q + k;
        if (p >= P) break;
        const int y = p / w;
        const bool b = bit(y, p - y * w);
        parent[p] = b ? p : -1;
        local += b;
      }
    }
  }
  if (cc_block_sum(local, s_i) == 0) {     // np.sum(binary) == 0 -> [0, 0]
    if (tid == 0) { out[plane * 2] = 0; out[plane * 2 + 1] = 0; }
    return;
  }
  if constexpr (PRE) {
    const int nk = stats[plane].ncand;
    if (nk >= 1 && nk <= CC_KFAST) {
      // fast finish: the candidates' values are compacted (cc_scatter), their chunk
      // maxima known (cc_count); exact sums in label (root) order, first max kept
      const CcChunk* pc = ck + (size_t)plane * chunks;
      int order[CC_KFAST], tot[CC_KFAST], base[CC_KFAST];
      for (int k = 0; k < nk; ++k) order[k] = k;
      for (int i = 1; i < nk; ++i)
        for (int j = i; j > 0 && stats[plane].cand[order[j - 1]] > stats[plane].cand[order[j]]; --j) {
          const int t = order[j]; order[j] = order[j - 1]; order[j - 1] = t;
        }
      for (int k = 0, acc = 0; k < nk; ++k) {
        int t = 0;
        for (int c = tid; c < chunks; c += CC_NT) t += pc[c].count[k];
        tot[k] = cc_block_sum(t, s_i);
        base[k] = acc;
        acc += tot[k];
      }
      int bestk = -1;
      double bestsum = 0.0;
      for (int q = 0; q < nk; ++q) {
        const int k = order[q];
        const double sum = np_sum_block(vals + base[k], tot[k],
                                        bsum_all ? bsum_all + ((size_t)plane * CC_KFAST + k) * maxb : nullptr);
        if (bestk < 0 || sum > bestsum) { bestsum = sum; bestk = k; }   // first max
      }
      double bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int c = tid; c < chunks; c += CC_NT)
        if (pc[c].count[bestk] > 0) cc_pick(bv, bi, pc[c].bestv[bestk], pc[c].besti[bestk]);
      const int pbest = cc_block_argmax(bv, bi, s_d, s_i);
      if (tid == 0) {
        out[plane * 2] = pbest % w;
        out[plane * 2 + 1] = pbest / w;
      }
      return;
    }
  }
  if constexpr (!PRE) {
    __threadfence_block();
    __syncthreads();
    // union over the 4 raster-earlier neighbours (8-connectivity)
    for (int p = tid; p < P; p += CC_NT) {
      if (parent[p] < 0) continue;
      const int y = p / w, x = p - y * w;
      if (x > 0 && bit(y, x - 1)) uf_union(parent, p, p - 1);
      if (y > 0) {
        if (x > 0 && bit(y - 1, x - 1)) uf_union(parent, p, p - w - 1);
        if (bit(y - 1, x)) uf_union(parent, p, p - w);
        if (x + 1 < w && bit(y - 1, x + 1)) uf_union(parent, p, p - w + 1);
      }
    }
    __threadfence();
    __syncthreads();
    for (int p = tid; p < P; p += CC_NT)
      if (ld_parent(parent, p) >= 0)
        __hip_atomic_store(parent + p, uf_root(parent, p), __ATOMIC_RELAXED, UfScope<PT>::v);
    __threadfence();
    __syncthreads();
  }
  // np.argmax over the components' np.sum (hand.py:68-69): only components whose sum
  // can be the maximum need numpy's exact pairwise order.  An order-free fp64 sum per
  // root (register-aggregated atomics; relative error < 1e-12 for these sizes) finds
  // the maximum M; the components with approx >= M*(1-1e-9) -- in practice one -- are
  // the candidates, and only they are summed exactly, in label (= root raster) order,
  // first max kept.  Sums are of values > thre > 0.
  if constexpr (!PRE) {
    for (int p = tid; p < P; p += CC_NT) vals[p] = 0.0;
    __threadfence_block();
    __syncthreads();
    const int per = (P + CC_NT - 1) / CC_NT;
    cc_root_sums(parent, map, vals, tid * per, min(P, (tid + 1) * per));
    __threadfence();
    __syncthreads();
  }
  if constexpr (PRE) {
    if (tid == 0) s_ncand = stats[plane].ncand;
    if (tid < MAXC) s_cand[tid] = stats[plane].cand[tid];
  } else {
    double m = -INFINITY;
    for (int q = tid * CC_RUN; q < P; q += CC_NT * CC_RUN) {
#pragma unroll
      for (int k = 0; k < CC_RUN; ++k) {
        const int p = q + k;
        if (p < P && parent[p] == p) m = fmax(m, vals[p]);
      }
    }
    const double thr_c = cc_block_max(m, s_d) * (1.0 - 1e-9);
    if (tid == 0) s_ncand = 0;
    __syncthreads();
    for (int q = tid * CC_RUN; q < P; q += CC_NT * CC_RUN) {
#pragma unroll
      for (int k = 0; k < CC_RUN; ++k) {
        const int p = q + k;
        if (p < P && parent[p] == p && vals[p] >= thr_c) {
          const int slot = atomicAdd(&s_ncand, 1);
          if (slot < MAXC) s_cand[slot] = p;
        }
      }
    }
  }
  __syncthreads();
  const bool all_roots = s_ncand > MAXC;   // pathological ties: every component, exactly
  if (tid == 0) {
    if (!all_roots)                        // label order = root raster order
      for (int i = 1; i < s_ncand; ++i) {
        const int v = s_cand[i];
        int j = i - 1;
        while (j >= 0 && s_cand[j] > v) { s_cand[j + 1] = s_cand[j]; --j; }
        s_cand[j + 1] = v;
      }
    s_best_root = -1;
    s_best_sum = 0.0;
  }
  __syncthreads();
  const int ncand = s_ncand;
  for (int ci = 0, r0 = 0; all_roots ? r0 < P : ci < ncand; ++ci) {
    int root;
    if (all_roots) {
      // next root (parent[r] == r) at or after r0, found cooperatively
      int cand = 0x7fffffff;
      for (int p = r0 + tid; p < P; p += CC_NT)
        if (parent[p] == p) { cand = p; break; }
      root = cc_block_min(cand, s_i);
      if (root == 0x7fffffff) break;
      r0 = root + 1;
    } else {
      root = s_cand[ci];
    }
    // compact this component's values in raster order
    int base = 0;
    for (int c0 = root; c0 < P; c0 += CC_NT * CC_RUN) {
      const int q0 = c0 + tid * CC_RUN;
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < CC_RUN; ++k) cnt += (q0 + k < P && parent[q0 + k] == root) ? 1 : 0;
      int total;
      int o = base + cc_block_scan(cnt, s_i, total) - cnt;
#pragma unroll
      for (int k = 0; k < CC_RUN; ++k)
        if (q0 + k < P && parent[q0 + k] == root) vals[o++] = map[q0 + k];
      base += total;
    }
    __threadfence_block();
    __syncthreads();
    const double sum = np_sum_block(vals, base);
    if (tid == 0 && (s_best_root < 0 || sum > s_best_sum)) { s_best_sum = sum; s_best_root = root; }   // first max
    __syncthreads();
  }
  // util.npmax on map_ori with the other labels zeroed: first raster-order maximum
  const int best = s_best_root;
  double bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int q = tid * CC_RUN; q < P; q += CC_NT * CC_RUN) {
#pragma unroll
    for (int k = 0; k < CC_RUN; ++k) {
      const int p = q + k;
      if (p < P) cc_pick(bv, bi, parent[p] == best ? map[p] : 0.0, p);
    }
  }
  const int pbest = cc_block_argmax(bv, bi, s_d, s_i);
  if (tid == 0) {
    out[plane * 2] = pbest % w;       // [x, y]
    out[plane * 2 + 1] = pbest / w;
  }
}

// (also zeroes the post's two list counters z0, z1, z16 16-byte words at zb and y16 at yb -- one
// launch instead of four memsets)
__global__ void init_records_kernel(char* result, isl_layout lay, int n, int nlimbs, int* z0 = nullptr,
                                    int* z1 = nullptr, uint4* zb = nullptr, long long z16 = 0,
                                    uint4* yb = nullptr, long long y16 = 0) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f == 0) {
    if (z0) *z0 = 0;
    if (z1) *z1 = 0;
  }
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = f; i < z16; i += stride) zb[i] = make_uint4(0u, 0u, 0u, 0u);
  for (long long i = f; i < y16; i += stride) yb[i] = make_uint4(0u, 0u, 0u, 0u);
  if (f >= n) return;
  char* rec = result + (size_t)f * lay.record_bytes;
  *(int*)(rec + lay.status) = ISL_OK;
  for (int k = 0; k < 32; ++k) ((int*)(rec + lay.n_conns))[k] = k < nlimbs ? 0 : -1;
  *(int*)(rec + lay.n_rows) = 0;
}

// ---------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------

static inline long long al8(long long x) { return (x + 7) / 8 * 8; }


}  // namespace isl

using namespace isl;

extern "C" int isl_body_layout(int model_kind, const isl_caps* caps, isl_layout* out) {
  if (!caps || !out || (model_kind != ISL_BODY25 && model_kind != ISL_COCO)) {
    set_error("isl_body_layout: bad argument");
    return ISL_E_ARG;
  }
  const int njoint = model_kind == ISL_BODY25 ? 26 : 19;
  const int nlimbs = model_kind == ISL_BODY25 ? 24 : 19;
  long long o = 0;
  out->status = o; o += 8;
  out->n_peaks = o; o += 32 * 4;
  out->n_conns = o; o += 32 * 4;
  out->n_rows = o; o += 8;
  out->peaks = o = al8(o); o += (long long)(njoint - 1) * caps->max_peaks * 3 * 8;
  out->conns = o; o += (long long)nlimbs * caps->max_conns * 5 * 8;
  out->subset = o; o += (long long)caps->max_rows * (njoint + 1) * 8;
  out->record_bytes = al8(o);
  return ISL_OK;
}


static bool fused_blur_enabled() {
  const char* e = getenv("ISLPOSE_FUSED_BLUR");   // A/B switch (tests); default on
  return !(e && e[0] == '0');
}

// ISLPOSE_FUSED_WIDE=1: two-stage frames whose stage-2 scale needs the wide LDS window
// (Mode R at 368 x 656) resize on the fly in blur_nms too (A/B; per call).  Off by default:
// measured slower than materialising the planes (Mode R batch-32 post 1.54 -> 1.61 ms, batch
// 1 0.19 -> 0.22 ms, profiles/r03/wide/): two 72 KB blocks per CU and a 28-row horizontal
// pass per tile cost more than the 0.8 GB write and re-read.
#ifdef ISLPOSE_DEV
static bool fused_wide_enabled() {
  const char* e = getenv("ISLPOSE_FUSED_WIDE");
  return e && e[0] == '1';
}
#else
static bool fused_wide_enabled() { return false; }   // rejected: development build only
#endif

static int post_fail(int code, const char* msg) {
  set_error(msg);
  return code;
}

#define PHIP(expr)                                          \
  do {                                                      \
    hipError_t e_ = (expr);                                 \
    if (e_ != hipSuccess) {                                 \
      set_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
      return ISL_E_HIP;                                     \
    }                                                       \
  } while (0)

// planar resize of n*nch planes (see resize_sep_kernel); rows per tile sized to the LDS window
// bandmax (mode 1): also write the band maxima of the output planes (resize_sep_kernel BM) when
// the tiles align with the bands; *bm_done says whether they were written
static int resize_rows(const MapSrc& m) {   // output rows per resize tile
  int ty = RS_TY;
  if (!m.identity)
    while (ty > 1 && (ty - 1) * m.scy + 5.0 > (double)RS_MAXR) --ty;
  return ty;
}
// the band-maxima form of launch_resize runs (and so `need` may be given)
static bool resize_bm_v4(const MapSrc& m, int ow) {
  const char* v4e = getenv("ISLPOSE_RESIZE_V4");
  return !m.identity && ow % 4 == 0 && resize_rows(m) == 4 * BM_ROWS && !(v4e && v4e[0] == '0');
}
static int launch_resize(const MapSrc& m, int n, int nch, int oh, int ow, int mode, float div_f, void* out,
                         hipStream_t s, float* bandmax = nullptr, bool* bm_done = nullptr,
                         const unsigned char* need = nullptr) {
  const int ty = resize_rows(m);
  const long long ty_tiles = (oh + ty - 1) / ty;
  if (ty_tiles > 65535) return post_fail(ISL_E_ARG, "resize: output too tall");
  if (bm_done) *bm_done = false;
  // (ISLPOSE_RESIZE_V4=0: the one-column vertical pass everywhere; A/B, per call)
  const char* v4e = getenv("ISLPOSE_RESIZE_V4");
  const bool v4 = mode == 1 && !m.identity && ow % 4 == 0 && ty % 4 == 0 && !(v4e && v4e[0] == '0');
  if (bandmax && mode == 1 && ty % BM_ROWS == 0) {
    if (v4 && ty == 4 * BM_ROWS)
      hipLaunchKernelGGL((resize_sep_kernel<128, 4, 8, true, true>), dim3(n * nch, (unsigned)ty_tiles, (ow + 127) / 128),
                         dim3(128), 0, s, m, nch, oh, ow, ty, mode, div_f, out, bandmax, need);
    else if (need)
      return post_fail(ISL_E_ARG, "resize: `need` without the band-maxima form");
    else
      hipLaunchKernelGGL((resize_sep_kernel<128, 4, 8, true>), dim3(n * nch, (unsigned)ty_tiles, (ow + 127) / 128),
                         dim3(128), 0, s, m, nch, oh, ow, ty, mode, div_f, out, bandmax);
    PHIP(hipGetLastError());
    if (bm_done) *bm_done = true;
    return ISL_OK;
  }
  if (v4) {
    hipLaunchKernelGGL((resize_sep_kernel<128, 4, 8, false, true>), dim3(n * nch, (unsigned)ty_tiles, (ow + 127) / 128),
                       dim3(128), 0, s, m, nch, oh, ow, ty, mode, div_f, out);
    PHIP(hipGetLastError());
    return ISL_OK;
  }
  // 128-column blocks unless 256 pads less (it never does): fewer idle lanes (ow = 328: 384 vs
  // 512), and at equal padding (ow = 656) twice the resident blocks: Mode R batch-32 post
  // 1.51 / 1.49 -> 1.47 / 1.47 ms; 32 or 16 rows per block lost (profiles/r03/rsty/)
  // vertical pass unrolled by 4: Mode R batch-32 post -2.5 %, batch 1 -1.8 %; staging the
  // source window in LDS lost 20 %, 16 source rows in flight instead of 8 gained nothing
  // (tools/resize_ab.py, profiles/r04/r4d/resize_ab.json)
  if ((ow + 127) / 128 * 128 <= (ow + RS_TX - 1) / RS_TX * RS_TX)
    hipLaunchKernelGGL((resize_sep_kernel<128, 4>), dim3(n * nch, (unsigned)ty_tiles, (ow + 127) / 128), dim3(128), 0, s,
                       m, nch, oh, ow, ty, mode, div_f, out);
  else
    hipLaunchKernelGGL((resize_sep_kernel<RS_TX, 4>), dim3(n * nch, (unsigned)ty_tiles, (ow + RS_TX - 1) / RS_TX),
                       dim3(RS_TX), 0, s, m, nch, oh, ow, ty, mode, div_f, out);
  PHIP(hipGetLastError());
  return ISL_OK;
}


// Low-res map of scale s: caller NCHW array or the net's arena output.
static int low_src(isl_net* net, const float* p, int which, int n, int C, int h8, int w8, MapSrc* m) {
  if (p) {
    m->base = p;
    m->xs = 1; m->ys = w8; m->cstr = (long long)h8 * w8; m->fs = (long long)C * h8 * w8;
    m->cshift = 30; m->cbig = 0;
    m->sh = h8; m->sw = w8;
    return ISL_OK;
  }
  const int rc = net_low_res(net, which, m);
  if (rc) return rc;
  if (m->sh != h8 || m->sw != w8) return post_fail(ISL_E_STATE, "arena output does not match the scale geometry");
  return ISL_OK;
}

#ifdef ISLPOSE_DEV
// ISLPOSE_TILE_PROF=1 (development build): the next blur launches stamp their tiles into a
// device buffer of `tiles` x 10 u64 (zeroed here); isl_dev_tile_prof copies it out
static unsigned long long* g_prof_buf = nullptr;
static size_t g_prof_tiles = 0;
static void tile_prof_arm(size_t tiles, hipStream_t s) {
  const char* e = getenv("ISLPOSE_TILE_PROF");
  unsigned long long* p = nullptr;
  if (e && e[0] == '1') {
    if (tiles > g_prof_tiles) {
      if (g_prof_buf) (void)hipFree(g_prof_buf);
      g_prof_buf = nullptr;
      if (hipMalloc(&g_prof_buf, tiles * 10 * 8) != hipSuccess) g_prof_buf = nullptr;
      g_prof_tiles = g_prof_buf ? tiles : 0;
    }
    if (g_prof_buf) (void)hipMemsetAsync(g_prof_buf, 0, tiles * 10 * 8, s);
    p = g_prof_buf;
  }
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tile_prof), &p, sizeof(p), 0, hipMemcpyHostToDevice, s);
}
// ISLPOSE_ASM_PROF=1 (development build): assemble_kernel stamps its phases per frame
static unsigned long long* g_asm_buf = nullptr;
static size_t g_asm_frames = 0;
static void asm_prof_arm(size_t frames, hipStream_t s) {
  const char* e = getenv("ISLPOSE_ASM_PROF");
  unsigned long long* p = nullptr;
  if (e && e[0] == '1') {
    if (frames > g_asm_frames) {
      if (g_asm_buf) (void)hipFree(g_asm_buf);
      g_asm_buf = nullptr;
      if (hipMalloc(&g_asm_buf, frames * 8 * 8) != hipSuccess) g_asm_buf = nullptr;
      g_asm_frames = g_asm_buf ? frames : 0;
    }
    p = g_asm_buf;
  }
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_asm_prof), &p, sizeof(p), 0, hipMemcpyHostToDevice, s);
}
extern "C" int isl_dev_asm_prof(void* host, size_t frames) {
  if (!g_asm_buf || frames > g_asm_frames) return ISL_E_ARG;
  return hipMemcpy(host, g_asm_buf, frames * 8 * 8, hipMemcpyDeviceToHost) == hipSuccess ? ISL_OK : ISL_E_HIP;
}
extern "C" int isl_dev_tile_prof(void* host, size_t tiles) {
  if (!g_prof_buf || tiles > g_prof_tiles) return ISL_E_ARG;
  return hipMemcpy(host, g_prof_buf, tiles * 10 * 8, hipMemcpyDeviceToHost) == hipSuccess ? ISL_OK : ISL_E_HIP;
}
#else
static void tile_prof_arm(size_t, hipStream_t) {}
static void asm_prof_arm(size_t, hipStream_t) {}
#endif

extern "C" int isl_body_post(isl_net* net, int n, int H, int W, int nscales, const isl_scale_geom* geom,
                             const float* const* d_paf, const float* const* d_heat, const isl_caps* caps,
                             void* d_result, void* stream) {
  if (!net || n <= 0 || H <= 0 || W <= 0 || nscales <= 0 || nscales > MAX_SCALES || !geom || !caps || !d_result)
    return post_fail(ISL_E_ARG, "isl_body_post: bad argument");
  const int kind = net_kind(net);
  if (kind != ISL_BODY25 && kind != ISL_COCO) return post_fail(ISL_E_ARG, "isl_body_post needs a body net");
  PHIP(hipSetDevice(net_device(net)));
  hipStream_t s = (hipStream_t)stream;
  const int njoint = kind == ISL_BODY25 ? 26 : 19, npaf = kind == ISL_BODY25 ? 52 : 38;
  const int nparts = njoint - 1, nlimbs = kind == ISL_BODY25 ? 24 : 19;
  isl_layout lay;
  int rc = isl_body_layout(kind, caps, &lay);
  if (rc) return rc;
  // ---- scratch plan ----
  const bool multi = nscales > 1;
  // single scale with the net input at frame size (one x8 resize): fuse resize + blur,
  // no full-resolution heat planes
  // single scale, two stages (Mode R on large frames: 184 x 327 -> 1080 x 1920): the
  // second resize is a strong upsampling whose full-resolution planes cost more HBM
  // traffic than the on-the-fly resize; fused too when a blur tile's source window fits
  // the LDS window (~1/5.2 and below; at 368 x 656, scale 1/2, it does not)
  // (the wide window takes stage-2 scales down to ~1/2: Mode R at 368 x 656)
  auto window_fits = [&](int rows, int cols) {
    return 41.0 * geom[0].valid_h / H + 6.0 <= rows && 217.0 * geom[0].valid_w / W + 6.0 <= cols;
  };
  const bool two = !multi && !(geom[0].valid_h == H && geom[0].valid_w == W);
  const bool fuse2_small = two && window_fits(NMS_SRC_ROWS, NMS_SRC_COLS);
  const bool fuse2 = two && (fuse2_small || (window_fits(NMS_WSRC_ROWS, NMS_WSRC_COLS) && fused_wide_enabled()));
  const bool wide = fuse2 && !fuse2_small;
  const bool fused = !multi && ((geom[0].valid_h == H && geom[0].valid_w == W) || fuse2) && fused_blur_enabled();
  const size_t heat_bytes = fused ? 0 : (size_t)n * nparts * H * W * (multi ? 8 : 4);
  size_t mid_bytes = 0;
  for (int si = 0; si < nscales; ++si) {
    const isl_scale_geom& g = geom[si];
    if (!(g.valid_h == H && g.valid_w == W)) mid_bytes += (size_t)n * g.valid_h * g.valid_w * nparts * 4;
  }
  const int words = (W + 63) / 64;
  const size_t mask_bytes = (size_t)n * nparts * H * words * 8;
  const size_t pair_bytes = (size_t)n * nlimbs * caps->max_pairs * (8 + 4 + 4);
  const size_t used_bytes = (size_t)n * nlimbs * 2 * caps->max_peaks;
  const size_t n_tiles_all = (size_t)((W + NMS_TX - 1) / NMS_TX) * ((H + NMS_TY - 1) / NMS_TY) * n * nparts;
  // ISLPOSE_BLUR_LIST=0: the band-maxima early out inside every tile's block instead of a live
  // list (A/B; per call)
  const char* ble = getenv("ISLPOSE_BLUR_LIST");
  const bool band_list = !(ble && ble[0] == '0');
  // single scale, materialised planes: the band maxima of the final resize (blur early out)
  // (ISLPOSE_BLUR_BANDS=0: without, A/B; read per call)
  const char* bme = getenv("ISLPOSE_BLUR_BANDS");
  const bool bands_on = !(bme && bme[0] == '0');
  const size_t bm_bytes = (!fused && !multi && bands_on) ? (size_t)n * nparts * ((H + BM_ROWS - 1) / BM_ROWS) * words * 4 : 0;
  const size_t live_bytes = (fused || (bm_bytes && band_list)) ? (n_tiles_all + 1) * sizeof(int) : 0;
  const size_t amb_bytes = (n_tiles_all + 1) * sizeof(int);   // the filter's undecided tiles
  // two-stage frames: stage-2 tiles that no live window reads are skipped (stage2_need_kernel;
  // ISLPOSE_RESIZE_SKIP=0 off, A/B, per call).  bm1: the stage-1 planes' band maxima
  const char* rse = getenv("ISLPOSE_RESIZE_SKIP");
  const isl_scale_geom& g0 = geom[0];
  MapSrc m2probe{};
  m2probe.identity = 0;
  m2probe.scy = 1.0 / ((double)H / g0.valid_h);
  MapSrc m1probe{};
  m1probe.identity = 0;
  m1probe.scy = 1.0 / 8.0;
  const bool skip2 = !fused && !multi && two && bm_bytes && band_list && !(rse && rse[0] == '0') &&
                     resize_bm_v4(m1probe, g0.valid_w) && resize_bm_v4(m2probe, W);
  const int ty2 = resize_rows(m2probe), ry_tiles = (H + ty2 - 1) / ty2, rx_tiles = (W + 127) / 128;
  const size_t bm1_bytes = skip2 ? (size_t)n * nparts * ((g0.valid_h + BM_ROWS - 1) / BM_ROWS) * ((g0.valid_w + 63) / 64) * 4 : 0;
  const size_t lmid_bytes = skip2 ? n_tiles_all : 0;
  const size_t need_bytes = skip2 ? (size_t)n * nparts * ry_tiles * rx_tiles : 0;
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t total = up(heat_bytes) + up(mid_bytes) + up(mask_bytes) + up(pair_bytes) + up(used_bytes) +
                       up(live_bytes) + up(bm_bytes) + up(amb_bytes) + up(bm1_bytes) + up(lmid_bytes) +
                       up(need_bytes);
  char* base = (char*)net_scratch(net, total);
  if (!base) return ISL_E_HIP;
  char* heat = base;
  char* mid = heat + up(heat_bytes);
  unsigned long long* mask = (unsigned long long*)(mid + up(mid_bytes));
  char* pairs = (char*)mask + up(mask_bytes);
  unsigned char* used = (unsigned char*)(pairs + up(pair_bytes));
  int* live_count = (int*)(used + up(used_bytes));
  int* live = live_count + 1;
  float* bandmax = bm_bytes ? (float*)((char*)live_count + up(live_bytes)) : nullptr;
  int* amb = (int*)((char*)live_count + up(live_bytes) + up(bm_bytes));
  float* bm1 = skip2 ? (float*)((char*)amb + up(amb_bytes)) : nullptr;
  unsigned char* live_mid = skip2 ? (unsigned char*)bm1 + up(bm1_bytes) : nullptr;
  unsigned char* need = skip2 ? live_mid + up(lmid_bytes) : nullptr;
  bool bm_done = false;

  // (amb[0]: the filter's list count; need: zeroed here for stage2_need_kernel; the peak mask
  // too when the blur runs over a live list, which writes the live tiles' words only)
  const long long need16 = (long long)(up(need_bytes) / 16);
  const long long mask16 = live_bytes ? (long long)(up(mask_bytes) / 16) : 0;
  hipLaunchKernelGGL(init_records_kernel,
                     dim3(std::max<long long>((n + 255) / 256, std::min<long long>((need16 + mask16 + 1023) / 1024, 2048))),
                     dim3(256), 0, s, (char*)d_result, lay, n, nlimbs, live_bytes ? live_count : nullptr, amb,
                     (uint4*)need, need16, (uint4*)mask, mask16);
  PHIP(hipGetLastError());

  GroupArgs ga;
  memset(&ga, 0, sizeof(ga));
  MapSrcN fin;                      // multi-scale: every scale's final-resolution heat source
  char* midp = mid;
  MapSrc fused_src{};
  const float div_f = (float)nscales;
  for (int si = 0; si < nscales; ++si) {
    const isl_scale_geom& g = geom[si];
    const int h8 = g.net_h / 8, w8 = g.net_w / 8;
    MapSrc lh, lp;
    if ((rc = low_src(net, d_heat ? d_heat[si] : nullptr, 1, n, njoint, h8, w8, &lh))) return rc;
    if ((rc = low_src(net, d_paf ? d_paf[si] : nullptr, 0, n, npaf, h8, w8, &lp))) return rc;
    // stage 1: cv2.resize(fx=fy=8) -> (h8*8, w8*8); crop to (valid_h, valid_w)
    lh.dh = lp.dh = h8 * 8; lh.dw = lp.dw = w8 * 8;
    lh.scy = lh.scx = lp.scy = lp.scx = 1.0 / 8.0;
    lh.cn = njoint; lp.cn = npaf;
    lh.identity = lp.identity = 0;
    const bool two_stage = !(g.valid_h == H && g.valid_w == W);
    MapSrc fh, fp;   // final-resolution sources
    if (two_stage) {
      float* mh = (float*)midp;
      midp += (size_t)n * g.valid_h * g.valid_w * nparts * 4;
      bool bm1_done = false;
      if ((rc = launch_resize(lh, n, nparts, g.valid_h, g.valid_w, 1, 1.f, mh, s, skip2 ? bm1 : nullptr, &bm1_done)))
        return rc;
      if (skip2 && !bm1_done) return post_fail(ISL_E_HIP, "body post: stage-1 band maxima not written");
      // the PAF's stage 1 is not materialised: limb_kernel samples both stages on demand
      // stage 2: cv2.resize(crop, (W, H)): inv_scale = W / valid_w, scale = 1 / inv_scale
      auto stage2 = [&](MapSrc& m, const float* p, int C, int cn) {
        m.base = p; m.xs = 1; m.ys = g.valid_w; m.cstr = (long long)g.valid_h * g.valid_w;
        m.fs = (long long)C * g.valid_h * g.valid_w;
        m.cshift = 30; m.cbig = 0;
        m.sh = g.valid_h; m.sw = g.valid_w; m.dh = H; m.dw = W;
        m.scy = 1.0 / ((double)H / g.valid_h); m.scx = 1.0 / ((double)W / g.valid_w);
        m.cn = cn; m.identity = 0;
      };
      stage2(fh, mh, nparts, njoint);
      stage2(fp, nullptr, npaf, npaf);
      ga.paf1[si] = lp;
      ga.paf_nested[si] = 1;
    } else {
      fh = lh;
      fp = lp;
    }
    if (fused) fused_src = fh;   // no full-resolution heat: blur_nms resizes on the fly
    else if (multi) fin.m[si] = fh;   // every scale's final resize, one fp64 pass below
    else {
      if (skip2) {
        const int tx = (W + NMS_TX - 1) / NMS_TX, tyl = (H + NMS_TY - 1) / NMS_TY, nt = (int)n_tiles_all;
        hipLaunchKernelGGL(stage2_need_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, fh, (const float*)bm1, H, W, tx,
                           tyl, nt, 0.1, ty2, ry_tiles, rx_tiles, live_mid, need);
        PHIP(hipGetLastError());
      }
      if ((rc = launch_resize(fh, n, nparts, H, W, 1, div_f, heat, s, bandmax, &bm_done, need))) return rc;
    }
    ga.paf[si] = fp;
  }
  if (multi) {
    // heatmap_avg += heatmap_avg + heatmap / len(m) over the scales (body.py:80, the
    // doubling quirk) in fp64 registers, one store (resize_acc_kernel)
    int ty = RA_TY;
    for (int si = 0; si < nscales; ++si)
      if (!fin.m[si].identity)
        while (ty > 1 && (ty - 1) * fin.m[si].scy + 5.0 > (double)RS_MAXR) --ty;
    const long long ty_tiles = (H + ty - 1) / ty;
    if (ty_tiles > 65535) return post_fail(ISL_E_ARG, "body post: frame too tall");
    hipLaunchKernelGGL(resize_acc_kernel, dim3(n * nparts, (unsigned)ty_tiles, (W + RS_TX - 1) / RS_TX), dim3(RS_TX),
                       0, s, fin, nscales, nparts, H, W, ty, div_f, 1, (double*)heat);
    PHIP(hipGetLastError());
  }
  // blur + NMS (body.py:86-100)
  dim3 gb((W + NMS_TX - 1) / NMS_TX, (H + NMS_TY - 1) / NMS_TY, n * nparts);
  tile_prof_arm((size_t)gb.x * gb.y * gb.z, s);
  const int tx = (int)gb.x, tyl = (int)gb.y;
  if (multi) {
    if ((rc = launch_blur<double, false>(gb, s, (const double*)heat, H, W, words, mask, 0.1, 0, MapSrc{}, 0, nullptr,
                                         nullptr, tx, tyl, nullptr, amb, true)))
      return rc;
  } else if (fused) {
    // live-tile list (low-res bound), then the fused blur over live tiles only
    const int n_tiles = (int)(gb.x * gb.y * gb.z);
    // (mask, live_count: zeroed by init_records_kernel)
    const dim3 tl((n_tiles + TL_TILES - 1) / TL_TILES);
    if (wide) {
#ifdef ISLPOSE_DEV
      hipLaunchKernelGGL((tile_live_kernel<NMS_WSRC_ROWS, NMS_WSRC_COLS>), tl, dim3(256), 0, s, fused_src, nparts, H, W,
                         tx, tyl, n_tiles, 0.1, live, live_count);
      PHIP(hipGetLastError());
      if ((rc = launch_blur<float, true, NMS_WSRC_ROWS, NMS_WSRC_COLS>(
               dim3(std::min((n_tiles + 7) / 8 * 8, 256 * 4)), s, (const float*)nullptr, H, W, words, mask, 0.1, 0, fused_src, nparts,
               live, live_count, tx, tyl, nullptr, amb, true)))
        return rc;
#endif
    } else {
      hipLaunchKernelGGL((tile_live_kernel<NMS_SRC_ROWS, NMS_SRC_COLS>), tl, dim3(256), 0, s, fused_src, nparts, H, W,
                         tx, tyl, n_tiles, 0.1, live, live_count);
      PHIP(hipGetLastError());
      if ((rc = launch_blur<float, true>(dim3(std::min((n_tiles + 7) / 8 * 8, 256 * 8)), s, (const float*)nullptr, H, W, words, mask,
                                         0.1, 0, fused_src, nparts, live, live_count, tx, tyl, nullptr, amb, true)))
        return rc;
    }
  } else if (bm_done && band_list) {
    // live-tile list (the band maxima), then the blur over live tiles only
    const int n_tiles = (int)(gb.x * gb.y * gb.z);
    // (mask, live_count: zeroed by init_records_kernel)
    hipLaunchKernelGGL(band_live_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, s, (const float*)bandmax, H, W,
                       words, tx, tyl, n_tiles, 0.1, live, live_count, (const unsigned char*)live_mid);
    PHIP(hipGetLastError());
    if ((rc = launch_blur<float, false>(dim3(std::min((n_tiles + 7) / 8 * 8, 256 * 8)), s, (const float*)heat, H, W, words, mask,
                                        0.1, 0, MapSrc{}, 0, live, live_count, tx, tyl, nullptr, amb, true)))
      return rc;
  } else if ((rc = launch_blur<float, false>(gb, s, (const float*)heat, H, W, words, mask, 0.1, 0, MapSrc{}, 0, nullptr,
                                             nullptr, tx, tyl, bm_done ? (const float*)bandmax : nullptr, amb, true))) {
    return rc;
  }
  PHIP(hipGetLastError());
  if (multi)
    hipLaunchKernelGGL((compact_kernel<double, false>), dim3(nparts, n), dim3(256), 0, s, mask, (const double*)heat,
                       nparts, H, W, words, (char*)d_result, lay, caps->max_peaks, MapSrc{});
  else if (fused)
    hipLaunchKernelGGL((compact_kernel<float, true>), dim3(nparts, n), dim3(256), 0, s, mask, (const float*)nullptr,
                       nparts, H, W, words, (char*)d_result, lay, caps->max_peaks, fused_src);
  else
    hipLaunchKernelGGL((compact_kernel<float, false>), dim3(nparts, n), dim3(256), 0, s, mask, (const float*)heat,
                       nparts, H, W, words, (char*)d_result, lay, caps->max_peaks, MapSrc{});
  PHIP(hipGetLastError());
  ga.nscales = nscales;
  ga.div_f = div_f;
  ga.H = H; ga.W = W;
  ga.model = kind; ga.njoint = njoint; ga.nlimbs = nlimbs;
  ga.max_peaks = caps->max_peaks; ga.max_pairs = caps->max_pairs; ga.max_conns = caps->max_conns;
  ga.max_rows = caps->max_rows;
  ga.lay = lay;
  ga.result = (char*)d_result;
  const size_t slots = (size_t)n * nlimbs;
  ga.pair_score = (double*)pairs;
  ga.pair_keep = (int*)(pairs + slots * caps->max_pairs * 8);
  ga.order = ga.pair_keep + slots * caps->max_pairs;
  ga.used = used;
  {   // ISLPOSE_LIMB_LDS=0: large pair sets on the per-thread pair loop (A/B and tests; read per call)
    const char* e = getenv("ISLPOSE_LIMB_LDS");
    ga.limb_lds = !(e && e[0] == '0');
  }
  // a frame per call: the scoring over Z blocks per limb (MODE 1), then ranks and matches (MODE 2);
  // ISLPOSE_LIMB_SPLIT=0: one block per limb (A/B; read per call)
  const char* lse = getenv("ISLPOSE_LIMB_SPLIT");
  // ISLPOSE_LIMB_Z=z: z blocks per limb (A/B; read per call).  A 1080p frame's scoring: 10 / 32 /
  // 64 blocks per limb 70.7 / 34.5 / 40.5 us (profiles/r06/lk/lz/); each pair is scored whole
  // by one block, so the slicing changes no sum
  const char* lzs = getenv("ISLPOSE_LIMB_Z");
  const int lz = (lse && lse[0] == '0') || n * nlimbs >= 128 ? 1
                 : lzs ? std::max(1, std::min(64, atoi(lzs))) : std::max(1, std::min(32, 1024 / (n * nlimbs)));
  if (lz > 1) {
    hipLaunchKernelGGL(limb_kernel<1>, dim3(nlimbs, n, lz), dim3(256), 0, s, ga);
    hipLaunchKernelGGL(limb_kernel<2>, dim3(nlimbs, n), dim3(256), 0, s, ga);
  } else {
    hipLaunchKernelGGL(limb_kernel<0>, dim3(nlimbs, n), dim3(256), 0, s, ga);
  }
  PHIP(hipGetLastError());
  const int asm_lds = caps->max_rows <= ASM_LDS_ROWS;
  // (the connection cache takes what is left of 64 KB of dynamic LDS, up to ASM_CONN_CACHE)
  const size_t sub_lds = asm_lds ? (size_t)caps->max_rows * (njoint + 1) * 8 : 0;
  const int conn_cap = (int)std::min<size_t>(ASM_CONN_CACHE, sub_lds < 65536 ? (65536 - sub_lds) / 40 : 0);
  asm_prof_arm((size_t)n, s);
  // ISLPOSE_ASM_REG=0: the table merge only (A/B; read per call)
  const char* are = getenv("ISLPOSE_ASM_REG");
  const int use_reg = !(are && are[0] == '0');
  if (kind == ISL_BODY25) {
    if (asm_lds)
      hipLaunchKernelGGL((assemble_kernel<true, ISL_BODY25>), dim3(n), dim3(64), sub_lds + (size_t)conn_cap * 40, s, ga,
                         conn_cap, use_reg);
    else
      hipLaunchKernelGGL((assemble_kernel<false, ISL_BODY25>), dim3(n), dim3(64), (size_t)conn_cap * 40, s, ga, conn_cap,
                         use_reg);
  } else {
    if (asm_lds)
      hipLaunchKernelGGL((assemble_kernel<true, ISL_COCO>), dim3(n), dim3(64), sub_lds + (size_t)conn_cap * 40, s, ga,
                         conn_cap, use_reg);
    else
      hipLaunchKernelGGL((assemble_kernel<false, ISL_COCO>), dim3(n), dim3(64), (size_t)conn_cap * 40, s, ga, conn_cap,
                         use_reg);
  }
  PHIP(hipGetLastError());
  return ISL_OK;
}

// scratch bytes of one hand post of n crops of h x w (layout: hand_post_launch)
static size_t hand_post_bytes(int n, int h, int w, int nscales, const isl_scale_geom* geom) {
  const int nparts = 21;
  const size_t P = (size_t)h * w;
  const int words = (w + 63) / 64;
  size_t mid_bytes = 0;   // every scale's intermediate stays until the fused average
  for (int si = 0; si < nscales; ++si)
    if (!(geom[si].valid_h == h && geom[si].valid_w == w))
      mid_bytes += (size_t)n * geom[si].valid_h * geom[si].valid_w * nparts * 4;
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t avg_bytes = (size_t)n * nparts * P * 8, mask_bytes = (size_t)n * nparts * h * words * 8;
  const size_t par_bytes = (size_t)n * nparts * P * 4, val_bytes = (size_t)n * nparts * P * 8;
  const size_t st_bytes = (size_t)n * nparts * sizeof(CcStats);
  const int cc_rows = std::max(1, CC_CHUNK / w), cc_chunks = (h + cc_rows - 1) / cc_rows;
  const size_t ck_bytes = (size_t)n * nparts * cc_chunks * sizeof(CcChunk);
  const size_t bs_bytes = (size_t)n * nparts * CC_KFAST * (P / 8192 + 1) * 8;
  const size_t amb_bytes = ((size_t)((w + NMS_TX - 1) / NMS_TX) * ((h + NMS_TY - 1) / NMS_TY) * n * nparts + 1) * 4;
  return up(avg_bytes) + up(mid_bytes) + up(mask_bytes) + up(par_bytes) + up(val_bytes) + up(st_bytes) + up(ck_bytes) +
         up(bs_bytes) + up(amb_bytes);
}

// the kernels of one hand post (hand.py:51-74) on stream s, scratch at base
// (hand_post_bytes); heat planes of scale si at d_heat[si] (NULL: the arena output)
static int hand_post_launch(isl_net* net, int n, int h, int w, int nscales, const isl_scale_geom* geom,
                            const float* const* d_heat, int64_t* d_peaks, hipStream_t s, char* base,
                            const float* const* mid_pre = nullptr) {
  const int nparts = 21, nch = 22;
  const size_t P = (size_t)h * w;
  const int words = (w + 63) / 64;
  size_t mid_bytes = 0;   // every scale's intermediate stays until the fused average
  for (int si = 0; si < nscales; ++si)
    if (!(geom[si].valid_h == h && geom[si].valid_w == w))
      mid_bytes += (size_t)n * geom[si].valid_h * geom[si].valid_w * nparts * 4;
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t avg_bytes = (size_t)n * nparts * P * 8, mask_bytes = (size_t)n * nparts * h * words * 8;
  const size_t par_bytes = (size_t)n * nparts * P * 4, val_bytes = (size_t)n * nparts * P * 8;
  const size_t st_bytes = (size_t)n * nparts * sizeof(CcStats);
  const int cc_rows = std::max(1, CC_CHUNK / w), cc_chunks = (h + cc_rows - 1) / cc_rows;
  double* avg = (double*)base;
  float* mid = (float*)(base + up(avg_bytes));
  unsigned long long* mask = (unsigned long long*)((char*)mid + up(mid_bytes));
  int* parent = (int*)((char*)mask + up(mask_bytes));
  double* vals = (double*)((char*)parent + up(par_bytes));
  CcStats* stats = (CcStats*)((char*)vals + up(val_bytes));
  CcChunk* cks = (CcChunk*)((char*)stats + up(st_bytes));
  double* bsum = (double*)((char*)cks + up((size_t)n * nparts * cc_chunks * sizeof(CcChunk)));
  int* amb = (int*)((char*)bsum + up((size_t)n * nparts * CC_KFAST * (P / 8192 + 1) * 8));
  const float div_f = (float)nscales;
  MapSrcN fin;                        // per scale: the resize that lands on the crop
  float* midp = mid;
  int ty = RA_TY;
  for (int si = 0; si < nscales; ++si) {
    const isl_scale_geom& g = geom[si];
    const int h8 = g.net_h / 8, w8 = g.net_w / 8;
    MapSrc lh;
    int rc = low_src(net, d_heat ? d_heat[si] : nullptr, 0, n, nch, h8, w8, &lh);
    if (rc) return rc;
    lh.dh = h8 * 8; lh.dw = w8 * 8; lh.scy = lh.scx = 1.0 / 8.0; lh.cn = nch; lh.identity = 0;
    MapSrc fh = lh;
    if (!(g.valid_h == h && g.valid_w == w)) {
      const float* mid_s = midp;
      if (mid_pre && mid_pre[si]) mid_s = mid_pre[si];   // stage 1 done for the whole crop batch
      else if ((rc = launch_resize(lh, n, nparts, g.valid_h, g.valid_w, 1, 1.f, midp, s))) return rc;
      fh.base = mid_s; fh.xs = 1; fh.ys = g.valid_w; fh.cstr = (long long)g.valid_h * g.valid_w;
      fh.fs = (long long)nparts * g.valid_h * g.valid_w;
      fh.cshift = 30; fh.cbig = 0;
      fh.sh = g.valid_h; fh.sw = g.valid_w; fh.dh = h; fh.dw = w;
      fh.scy = 1.0 / ((double)h / g.valid_h); fh.scx = 1.0 / ((double)w / g.valid_w);
      fh.cn = nch; fh.identity = 0;
      midp += (size_t)n * g.valid_h * g.valid_w * nparts;
    }
    fin.m[si] = fh;
    if (!fh.identity)   // rows per tile: every scale's source window fits the LDS rows
      while (ty > 1 && (ty - 1) * fh.scy + 5.0 > (double)RS_MAXR) --ty;
  }
  {
    const long long ty_tiles = (h + ty - 1) / ty;
    if (ty_tiles > 65535) return post_fail(ISL_E_ARG, "hand post: crop too tall");
    hipLaunchKernelGGL(resize_acc_kernel, dim3(n * nparts, (unsigned)ty_tiles, (w + RS_TX - 1) / RS_TX), dim3(RS_TX),
                       0, s, fin, nscales, nparts, h, w, ty, div_f, 0, avg);
    PHIP(hipGetLastError());
  }
  dim3 gb((w + NMS_TX - 1) / NMS_TX, (h + NMS_TY - 1) / NMS_TY, n * nparts);
  tile_prof_arm((size_t)gb.x * gb.y * gb.z, s);
  if (int rc = launch_blur<double, false>(gb, s, (const double*)avg, h, w, words, mask, 0.05, 1, MapSrc{}, 0, nullptr,
                                          nullptr, (int)gb.x, (int)gb.y, nullptr, amb))
    return rc;
  if (h * w <= CC_LDS_MAX) {
    static bool attr = false;
    if (!attr) {
      PHIP(hipFuncSetAttribute((const void*)hand_cc_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               CC_LDS_MAX * 4));
      attr = true;
    }
    hipLaunchKernelGGL((hand_cc_kernel<true, false>), dim3(n * nparts), dim3(CC_NT), (size_t)h * w * 4, s,
                       (const double*)avg, mask, h, w, words, parent, vals, nullptr, nullptr, 0, (long long*)d_peaks,
                       nullptr, 0);
  } else {
    if (w > CC_WMAX) return post_fail(ISL_E_ARG, "isl_hand_post: crop wider than 8192 px");
    const int rows = cc_rows, chunks = cc_chunks;
    const dim3 g(n * nparts * chunks);
    hipLaunchKernelGGL(cc_local_kernel, g, dim3(256), 0, s, mask, h, w, words, rows, chunks, parent, vals, stats);
    hipLaunchKernelGGL(cc_merge_kernel, g, dim3(256), 0, s, mask, h, w, words, rows, chunks, parent);
    hipLaunchKernelGGL(cc_find_kernel, g, dim3(256), 0, s, h, w, rows, chunks, parent, vals);
    hipLaunchKernelGGL(cc_sum_kernel, g, dim3(256), 0, s, (const double*)avg, h, w, rows, chunks, parent, vals, stats);
    hipLaunchKernelGGL(cc_stats_kernel, g, dim3(256), 0, s, h, w, rows, chunks, parent, vals, stats);
    hipLaunchKernelGGL(cc_cand_kernel, g, dim3(256), 0, s, h, w, rows, chunks, parent, vals, stats);
    hipLaunchKernelGGL(cc_count_kernel, g, dim3(256), 0, s, (const double*)avg, h, w, rows, chunks, parent, stats, cks);
    hipLaunchKernelGGL(cc_scatter_kernel, g, dim3(256), 0, s, (const double*)avg, h, w, rows, chunks, parent, stats, cks,
                       vals);
    const int maxb = (int)(P / 8192) + 1;
    hipLaunchKernelGGL(cc_bufsum_kernel, dim3(n * nparts, std::max(1, std::min(32, (maxb + 3) / 4))), dim3(256), 0, s,
                       stats, cks, chunks, (int)P, vals, bsum, maxb);
    hipLaunchKernelGGL((hand_cc_kernel<false, true>), dim3(n * nparts), dim3(CC_NT), 0, s, (const double*)avg, mask,
                       h, w, words, parent, vals, stats, cks, chunks, (long long*)d_peaks, bsum, maxb);
  }
  PHIP(hipGetLastError());
  return ISL_OK;
}

extern "C" int isl_hand_post(isl_net* net, int n, int h, int w, int nscales, const isl_scale_geom* geom,
                             const float* const* d_heat, int64_t* d_peaks, void* stream) {
  if (!net || n <= 0 || h <= 0 || w <= 0 || nscales <= 0 || nscales > MAX_SCALES || !geom || !d_peaks)
    return post_fail(ISL_E_ARG, "isl_hand_post: bad argument");
  if (net_kind(net) != ISL_HAND) return post_fail(ISL_E_ARG, "isl_hand_post needs the hand net");
  if (nscales > 1 && !d_heat) return post_fail(ISL_E_ARG, "isl_hand_post: maps required for several scales");
  PHIP(hipSetDevice(net_device(net)));
  char* base = (char*)net_scratch(net, hand_post_bytes(n, h, w, nscales, geom));
  if (!base) return ISL_E_HIP;
  return hand_post_launch(net, n, h, w, nscales, geom, d_heat, d_peaks, (hipStream_t)stream, base);
}

// Crops of different sizes in one call (HandEstimator.post_crops): crop i is a square of
// crop_w[i] px, geom[i * nscales + si] its scale geometries, its low-res maps crop i of
// d_heat[si] ([n,22,net_h/8,net_w/8]: every crop has the same net size per scale).  Each
// crop's kernel chain is small (21 planes), so the crops run on ISL_POST_LANES streams
// forked from `stream` and joined back into it, each lane with its own grow-only scratch.
extern "C" int isl_hand_post_crops(isl_net* net, int n, const int32_t* crop_w, int nscales,
                                   const isl_scale_geom* geom, const float* const* d_heat, int64_t* d_peaks,
                                   void* stream) {
  if (!net || n <= 0 || !crop_w || nscales <= 0 || nscales > MAX_SCALES || !geom || !d_heat || !d_peaks)
    return post_fail(ISL_E_ARG, "isl_hand_post_crops: bad argument");
  if (net_kind(net) != ISL_HAND) return post_fail(ISL_E_ARG, "isl_hand_post_crops needs the hand net");
  for (int i = 0; i < n; ++i) {
    if (crop_w[i] <= 0) return post_fail(ISL_E_ARG, "isl_hand_post_crops: bad crop size");
    for (int si = 0; si < nscales; ++si)
      if (geom[i * nscales + si].net_h != geom[si].net_h || geom[i * nscales + si].net_w != geom[si].net_w)
        return post_fail(ISL_E_ARG, "isl_hand_post_crops: crops differ in net size");
  }
  PHIP(hipSetDevice(net_device(net)));
  hipStream_t s = (hipStream_t)stream;
  PostLanes* L = net_post_lanes(net);
  if (!L) return ISL_E_HIP;
  const int nl = std::min(n, ISL_POST_LANES);
  // lane k takes crops k, k + nl, ...; size its scratch for the largest first, before any
  // launch of this call (a grown buffer is reallocated only once its lane has drained)
  for (int k = 0; k < nl; ++k) {
    size_t need = 0;
    for (int i = k; i < n; i += nl) need = std::max(need, hand_post_bytes(1, crop_w[i], crop_w[i], nscales, geom + (size_t)i * nscales));
    if (need > L->bytes[k]) {
      PHIP(hipStreamSynchronize(L->stream[k]));
      if (L->scratch[k]) PHIP(hipFree(L->scratch[k]));
      L->scratch[k] = nullptr;
      L->bytes[k] = 0;
      PHIP(hipMalloc(&L->scratch[k], need));
      L->bytes[k] = need;
    }
  }
  // Stage 1 of every scale (low-res x8 -> the net's valid size) for the whole crop batch, one
  // launch per scale on the caller's stream: every crop has the same net and valid size per
  // scale (round(s * 368) for square crops), so only the per-crop final resize onto the crop
  // is left to the lanes.  Scales whose valid size differs between crops stay per crop.
  float* mid_all[MAX_SCALES] = {};
  {
    size_t tot = 0, off[MAX_SCALES] = {};
    for (int si = 0; si < nscales; ++si) {
      bool same = true;
      for (int i = 1; i < n; ++i)
        same &= geom[i * nscales + si].valid_h == geom[si].valid_h && geom[i * nscales + si].valid_w == geom[si].valid_w;
      if (!same) continue;
      off[si] = tot + 1;   // + 1: "present"
      tot += ((size_t)n * 21 * geom[si].valid_h * geom[si].valid_w * 4 + 255) / 256 * 256;
    }
    if (tot) {
      // the maps' own buffer, not the net scratch (which isl_body_post / isl_hand_post on
      // other streams reuse): a previous call's lanes may still read it, so the writer waits
      // for their release event; growing it waits on the host, once per new maximum
      if (tot > L->mid_bytes) {
        if (L->mid) {
          if (L->mid_used) PHIP(hipEventSynchronize(L->mid_free));
          PHIP(hipFree(L->mid));
        }
        L->mid = nullptr;
        L->mid_bytes = 0;
        L->mid_used = false;
        PHIP(hipMalloc(&L->mid, tot));
        L->mid_bytes = tot;
      }
      if (L->mid_used) PHIP(hipStreamWaitEvent(s, L->mid_free, 0));
      char* base = (char*)L->mid;
      for (int si = 0; si < nscales; ++si) {
        if (!off[si]) continue;
        const isl_scale_geom& g = geom[si];
        const int h8 = g.net_h / 8, w8 = g.net_w / 8;
        MapSrc lh;
        int rc = low_src(net, d_heat[si], 0, n, 22, h8, w8, &lh);
        if (rc) return rc;
        lh.dh = h8 * 8; lh.dw = w8 * 8; lh.scy = lh.scx = 1.0 / 8.0; lh.cn = 22; lh.identity = 0;
        mid_all[si] = (float*)(base + off[si] - 1);
        if ((rc = launch_resize(lh, n, 21, g.valid_h, g.valid_w, 1, 1.f, mid_all[si], s))) return rc;
      }
    }
  }
  PHIP(hipEventRecord(L->fork, s));
  for (int k = 0; k < nl; ++k) PHIP(hipStreamWaitEvent(L->stream[k], L->fork, 0));
  for (int i = 0; i < n; ++i) {
    const int k = i % nl;
    const float* hp[MAX_SCALES];
    const float* mp[MAX_SCALES];
    for (int si = 0; si < nscales; ++si) {
      const isl_scale_geom& g = geom[si];
      hp[si] = d_heat[si] + (size_t)i * 22 * (g.net_h / 8) * (g.net_w / 8);
      mp[si] = mid_all[si] ? mid_all[si] + (size_t)i * 21 * g.valid_h * g.valid_w : nullptr;
    }
    const int rc = hand_post_launch(net, 1, crop_w[i], crop_w[i], nscales, geom + (size_t)i * nscales, hp,
                                    d_peaks + (size_t)i * 42, L->stream[k], (char*)L->scratch[k], mp);
    if (rc) return rc;
  }
  for (int k = 0; k < nl; ++k) {
    PHIP(hipEventRecord(L->join[k], L->stream[k]));
    PHIP(hipStreamWaitEvent(s, L->join[k], 0));
  }
  if (L->mid) {   // the lanes have joined: the stage-1 maps are free once s gets here
    PHIP(hipEventRecord(L->mid_free, s));
    L->mid_used = true;
  }
  return ISL_OK;
}

extern "C" int isl_debug_np_sum(const double* d_a, int64_t n, double* d_out, void* stream) {
  if (!d_a || !d_out || n <= 0 || n > (1ll << 30)) return post_fail(ISL_E_ARG, "isl_debug_np_sum: bad argument");
  hipLaunchKernelGGL(np_sum_debug_kernel, dim3(1), dim3(CC_NT), 0, (hipStream_t)stream, d_a, (int)n, d_out);
  PHIP(hipGetLastError());
  return ISL_OK;
}
