// 3x3 convolution (stride 1, pad 1) as Winograd F(2x2, 3x3) on the gfx950 FP16 matrix
// cores with split-fp16 (x3) products: the fp32-accurate arithmetic of conv_x3.hip on the
// 16 Winograd GEMMs, for the 3x3 layers of src/model.py:25-64 (make_layers /
// make_layers_Mconv) on chip-filling grids.
//
//   U = G g G^T   per (co, ci), host, double, x 2^s, split hi + lo     (pack_wino_f16)
//   V = B^T d B   per (tile, ci), in the kernel from the staged input, fp32, then split
//   M[xi] = sum_ci U[xi][co][ci] V[xi][ci][tile]   16 GEMMs, 3 fp16 MFMAs per product
//   Y = A^T M A   the 2x2 outputs of a tile, x 2^-s + bias, activation, range check
//
// 16 products per 2x2 outputs instead of 36: 2.25x fewer MFMAs than conv_x3_f16.  The
// transforms are exact-coefficient (0, +-1 for B and A; G's 1/2 in double on the host), so
// the accuracy class is that of conv_x3 (rel err ~1e-6 vs the fp64 forward).
//
// Round 1's split-fp16 Winograd (wino_x3.hip, development build) lost 1.3-1.8x: 4 waves
// of 64 channels computed all 16 V values of a tile per thread (184 VALU per (tile, channel),
// redone for every 64-channel block) into a single-buffered 128 KB step.  This kernel is built
// the other way round, so that no operand of the K loop is shared through LDS except the raw
// input:
//
//   * Block = 16 waves, wave w owns xi = w (one GEMM) for 64 output channels x 64 tiles
//     (2 x 2 accumulator tiles of 32 x 32, 64 registers).  U[xi] of the block is used by
//     that wave alone, so its A fragments go straight from L2 into registers (4 x 16 B per
//     lane and K step, loaded one step ahead) -- no LDS, no barrier for the filters.
//   * V[xi] is also used by that wave alone: the wave builds its B fragments itself from
//     the staged fp32 input, 4 pixels per (tile, channel) -- V[r][c] = (d[ra][ca] +
//     sc d[ra][cb]) + sr (d[rb][ca] + sc d[rb][cb]), B^T's rows having two nonzeros each --
//     3 fma + the split per value, 24 VALU per 8 values of a fragment.
//   * The raw input of a K step (a chunk pair) arrives by LDS-DMA, double-buffered, one
//     barrier per step.  The block's 64 tiles are consecutive in "band order" (a band = two
//     tile rows, walked column-pair by column-pair), so they touch at most two bands and the
//     staged run is 6 rows x (64 + 4) columns whatever the image width (26 KB per step).
//     Layout [chunk half h][channel quad q][row 6][column parity][34] x 16 B: the lanes of
//     a wave (consecutive band slots) read conflict-free ds_read_b128s (lane pairs 2k, 2k+1
//     differ by two rows = 32 banks, lane pairs by 16 B).
//   * Epilogue: the 16 waves' M tiles meet in LDS (two rounds of 32 channels, 128 KB), one
//     thread per (4 channels, tile) sums them in a fixed order into the 2x2 outputs.
//
// Per K step and CU (16 waves of 12 MFMAs): 1536 MFMA cycles against ~1000 LDS cycles
// (16 ds_read_b128 per wave), ~770 VALU cycles per SIMD and 64 KB of filters + 26 KB of
// input from L2.  Eligible launches (wino_f16_fits): 3x3, cout % 64 == 0, no fused pool or
// pooled-input staging, at least 32 tiles per row and > 1024 pixels per frame (no
// canonical K ranges: those layers keep conv_x3's batch-invariant sums).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "internal.h"

namespace isl {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct W2Args {
  const float* in;
  float* out;
  const f16x8* upk;             // [co_block][pair][xi][i 2][hi|lo][h][32] x 8 fp16 (pack_wino_f16)
  const float* bias;
  const float* slope;
  int* range_flag;
  long long in_fs, in_chs, out_fs, out_chs;   // frame / chunk strides (floats)
  float wscale_inv;             // 2^-s
  int in_pad, out_pad, H, W, TH, TW, pairs, cin_chunks, co_blocks, bpf, act, nblocks;
};

constexpr int RS = 34;                  // 16-byte units per staged (row, column parity): 68 columns
constexpr int QS = 6 * 2 * RS;          // per (chunk half, channel quad): 6 rows x 2 parities
constexpr int HS = 13 * 64;             // per chunk half: 2 quads (816 units) in 13 whole DMA pieces
constexpr int BUF = 32 * 64;            // 2048 units (32 KiB): 32 DMA pieces of 64 units, 2 per wave

// v = hi + lo for 4 fp32 values as dwords of 2 fp16 each (h01 = hi of v.x, v.y; ...): hi by the
// packed RNE conversion, lo = (f16)(v - (f32)hi) in one v_fma_mix per value (-1 * hi + v: the
// difference is exact in fp32, Sterbenz), written straight into its half of the dword -- the bits of
// conv_x3's x3_split8 in 1.5 instead of 3 VALU per value and no repacking moves.
__device__ __forceinline__ void split_dw(const f32x4& v, unsigned& h01, unsigned& h23, unsigned& l01, unsigned& l23) {
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h01) : "v"(v.x), "v"(v.y));
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(h23) : "v"(v.z), "v"(v.w));
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l01) : "v"(h01), "v"(v.x));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l01) : "v"(h01), "v"(v.y));
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l23) : "v"(h23), "v"(v.z));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l23) : "v"(h23), "v"(v.w));
}

// ABL (development build only, tools/convbench "w2" with ISLPOSE_W2_ABL): timing ablations --
// 1 no MFMAs, 2 no transform (no raw LDS reads, no VALU; constant B), 4 no filter loads, 8 no
// raw-input DMA, 16 no epilogue (the accumulators are folded into one store so that nothing
// upstream is dead code).  Wrong results; libislpose.so has ABL = 0 only.
template <int ABL>
__global__ void __launch_bounds__(512, 1) wino_f16(W2Args a) {
  // [0, 3 BUF): the raw-input ring; [0, 8192): the M exchange of the epilogue; then the epilogue's
  // bias and PReLU slopes (64 + 64 floats)
  __shared__ f32x4 smem[8192 + 32];

  // XCD-aware order (conv_x3): the channel blocks of a tile block, then neighbouring tile
  // blocks, on one XCD, so the staged input is read from one L2
  int bid = blockIdx.x;
  {
    const int nb = a.nblocks, q = nb >> 3, r = nb & 7, xcd = bid & 7, k = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int co_b = bid % a.co_blocks;
  const int rest = bid / a.co_blocks;
  const int fb = rest % a.bpf;
  const int n = rest / a.bpf;

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  // the epilogue's bias and slopes, staged once (read after the K loop's last barrier)
  if (tid < 64) {
    float* eb = (float*)(smem + 8192);
    eb[tid] = a.bias[co_b * 64 + tid];
    eb[64 + tid] = a.act == ACT_PRELU ? a.slope[co_b * 64 + tid] : 0.f;
  }

  // the block's 64 band slots s0 .. s0 + 63: band b = tile rows 2b, 2b + 1; slot u of a band =
  // tile (2b + (u & 1), u >> 1).  They lie in band ba and, past its end, in band bb = ba + 1
  // (TW >= 32); segment 0 = band ba's columns from txlo0, segment 1 = band bb's from 0
  const int BW = 2 * a.TW, s0 = fb * 64;
  const int ba = s0 / BW, bb = (s0 + 63) / BW;
  const bool two = bb > ba;
  const int txlo0 = (s0 - ba * BW) >> 1;
  const int txhi0 = two ? a.TW - 1 : (s0 + 63 - ba * BW) >> 1;
  const int w0 = 2 * (txhi0 - txlo0 + 1) + 2;                    // staged columns of segment 0
  const int w1 = two ? 2 * (((s0 + 63 - bb * BW) >> 1) + 1) + 2 : 0;
  const int Hp = a.H + 2 * a.in_pad, Wp = a.W + 2 * a.in_pad;
  const float* in_f = a.in + (size_t)n * a.in_fs;

  // Raw-input pieces of this wave: p = w + 8 e (e < 4), 64 units each.  Piece p stages chunk half
  // hp = p / 13 of the pair (13 pieces = 832 units per half: [q][row 6][parity][34] + 16 spare);
  // pieces 26 .. 31 are spare (they reload pixel 0 into the buffer's tail).  Lane unit -> (q, row,
  // parity, half column) -> the padded input pixel; rows / columns past the buffer, which only
  // feed discarded outputs, are clamped.  The chunk is wave-uniform: a uniform base plus a
  // 32-bit lane offset.
  int doff[4], dch[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int p = w + 8 * e;
    const int hp = p < 26 ? p / 13 : 0;
    const int u = (p - 13 * hp) * 64 + lane;             // unit within the half's region
    int t = u / RS;
    const int hc = u - t * RS;
    const int par = t & 1;
    t >>= 1;
    const int row = t % 6;
    const int qq = t / 6;
    const int v = 2 * hc + par;
    const bool s1 = v >= w0;
    const int vl = s1 ? v - w0 : v;
    const bool ok = p < 26 && qq < 2 && vl < (s1 ? w1 : w0);
    const int band = s1 ? bb : ba, txlo = s1 ? 0 : txlo0;
    const int rp = min(4 * band - 1 + row + a.in_pad, Hp - 1);
    const int cp = min(2 * txlo - 1 + vl + a.in_pad, Wp - 1);
    doff[e] = ok ? (rp * Wp + cp) * 8 + qq * 4 : 0;
    dch[e] = __builtin_amdgcn_readfirstlane(hp);
  }

  // This wave's two GEMMs: xi0 = 4 r + 2 cp, xi1 = xi0 + 1 (one row r of V, a column pair).
  // V[r][c] = (d[ra][ca] + sc d[ra][cb]) + sr (d[rb][ca] + sc d[rb][cb]); B^T rows: d0 - d2,
  // d1 + d2, d2 - d1, d1 - d3.  The row combination t[col] = d[ra][col] + sr d[rb][col] is
  // shared by the pair, over three column slots X, Y, Z: V(xi0) = tX - tY, V(xi1) = tY + sz tZ
  // (cp 0: columns 0, 2, 1, sz = +1 -- d0 - d2, d2 + d1; cp 1: columns 2, 1, 3, sz = -1 --
  // d2 - d1, d1 - d3): 6 pixels, 3 + 2 fma per channel for the two values, no selects.
  const int wr = w >> 1, cpr = w & 1;
  const int ra = wr == 0 ? 0 : wr == 2 ? 2 : 1, rb = wr == 3 ? 3 : wr == 2 ? 1 : 2;
  const float sr = wr == 1 ? 1.f : -1.f, sz = cpr ? -1.f : 1.f;
  const f32x4 srv = f32x4{sr, sr, sr, sr}, szv = f32x4{sz, sz, sz, sz};
  const int cX = cpr ? 2 : 0, cY = cpr ? 1 : 2, cZ = cpr ? 3 : 1;
  auto toff = [&](int row, int col) { return (row * 2 + (col & 1)) * RS + (col >> 1); };
  const int to_aX = toff(ra, cX), to_aY = toff(ra, cY), to_aZ = toff(ra, cZ);
  const int to_bX = toff(rb, cX), to_bY = toff(rb, cY), to_bZ = toff(rb, cZ);
  // per tile tile j the lane's unit base in a raw buffer (chunk half h, quad 0, row 2 typ, parity 0)
  int tb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int s = s0 + 32 * j + l32;
    const int band = s / BW, u = s - band * BW, tx = u >> 1, typ = u & 1;
    const int hc0 = band > ba ? (w0 >> 1) + tx : tx - txlo0;
    tb[j] = h * HS + 2 * typ * 2 * RS + hc0;
  }

  // Filters U[co_b][pair k][xi][i][hi|lo][h][32 co]: this wave's xi0 and xi1 are 8 contiguous
  // 1 KiB pieces (xi, i, hi|lo); lane offset h * 32 + co.  Loaded by inline asm (so the
  // compiler, which drains every outstanding load at the first use of an ordinary load while a
  // LDS-DMA is in flight, does not see them) and waited for with counted vmcnt below.
  const unsigned uvoff = (unsigned)lane * 16;
  auto load_a = [&](f16x8 (&A)[2][2][2], int k) __attribute__((always_inline)) {
    if constexpr ((ABL & 4) != 0) return;
    const f16x8* u0 = a.upk + ((size_t)(co_b * a.pairs + k) * 16 + 4 * wr + 2 * cpr) * 256;
    const f16x8* u1 = u0 + 256;
    asm volatile(
        "global_load_dwordx4 %0, %8, %9 offset:0\n\t"
        "global_load_dwordx4 %1, %8, %9 offset:1024\n\t"
        "global_load_dwordx4 %2, %8, %9 offset:2048\n\t"
        "global_load_dwordx4 %3, %8, %9 offset:3072\n\t"
        "global_load_dwordx4 %4, %8, %10 offset:0\n\t"
        "global_load_dwordx4 %5, %8, %10 offset:1024\n\t"
        "global_load_dwordx4 %6, %8, %10 offset:2048\n\t"
        "global_load_dwordx4 %7, %8, %10 offset:3072"
        : "=v"(A[0][0][0]), "=v"(A[0][0][1]), "=v"(A[0][1][0]), "=v"(A[0][1][1]), "=v"(A[1][0][0]),
          "=v"(A[1][0][1]), "=v"(A[1][1][0]), "=v"(A[1][1][1])
        : "v"(uvoff), "s"(u0), "s"(u1)
        : "memory");
  };
  // the raw input of pair k into ring slot sl (4 pieces of 64 units; counted by vmcnt)
  auto dma = [&](int k, int sl) __attribute__((always_inline)) {
    if constexpr ((ABL & 8) != 0) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = min(2 * k + dch[e], a.cin_chunks - 1);   // a missing odd chunk: zero filters
      const float* src = in_f + (size_t)ch * a.in_chs;
      __builtin_amdgcn_global_load_lds((const void*)(src + doff[e]),
                                       (__attribute__((address_space(3))) void*)(smem + sl * BUF + (w + 8 * e) * 64),
                                       16, 0, 0);
    }
  };

  f32x16 acc[2][2][2];   // [xi][i][j]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][i][j][r] = 0.f;
  // Range: a V value with |V| >= 65520 splits to an infinite hi, which makes every output it feeds
  // inf or NaN (a zero filter gives NaN too), so the epilogue's output check raises the range flag
  // (the host then recomputes on the fp32 kernels); |V| in [65504, 65520) splits exactly.

  // per tile tile j: both GEMMs' B fragments (the transform) from ring slot sl, then 12 MFMAs
  auto compute = [&](const f16x8 (&A)[2][2][2], int sl) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int b = tb[j] + sl * BUF;
      asm volatile("" : "+v"(b));   // the pixel addresses are formed per step (not held across it)
      // B fragments as dwords (2 fp16 each): [xi][hi|lo] x 4 dwords, quad Q in dwords 2Q, 2Q + 1
      unsigned Bd[2][2][4];
      if constexpr ((ABL & 2) != 0) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int hl = 0; hl < 2; ++hl)
#pragma unroll
            for (int d = 0; d < 4; ++d) Bd[x][hl][d] = 0x3c003c00u;
      } else {
        auto quad = [&](auto qc) __attribute__((always_inline)) {
          constexpr int Q = decltype(qc)::value;
          const f32x4 aX = smem[b + to_aX + Q * QS], aY = smem[b + to_aY + Q * QS], aZ = smem[b + to_aZ + Q * QS];
          const f32x4 bX = smem[b + to_bX + Q * QS], bY = smem[b + to_bY + Q * QS], bZ = smem[b + to_bZ + Q * QS];
          // (vector forms: each f32x4 op becomes two v_pk_*_f32 on the registers ds_read_b128 filled)
          const f32x4 tX = __builtin_elementwise_fma(srv, bX, aX);
          const f32x4 tY = __builtin_elementwise_fma(srv, bY, aY);
          const f32x4 tZ = __builtin_elementwise_fma(srv, bZ, aZ);
          const f32x4 v0 = tX - tY;
          const f32x4 v1 = __builtin_elementwise_fma(szv, tZ, tY);
          split_dw(v0, Bd[0][0][2 * Q], Bd[0][0][2 * Q + 1], Bd[0][1][2 * Q], Bd[0][1][2 * Q + 1]);
          split_dw(v1, Bd[1][0][2 * Q], Bd[1][0][2 * Q + 1], Bd[1][1][2 * Q], Bd[1][1][2 * Q + 1]);
        };
        quad(std::integral_constant<int, 0>{});
        quad(std::integral_constant<int, 1>{});
      }
      f16x8 Bh[2], Bl[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        Bh[x] = __builtin_bit_cast(f16x8, u32x4{Bd[x][0][0], Bd[x][0][1], Bd[x][0][2], Bd[x][0][3]});
        Bl[x] = __builtin_bit_cast(f16x8, u32x4{Bd[x][1][0], Bd[x][1][1], Bd[x][1][2], Bd[x][1][3]});
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr ((ABL & 1) != 0) continue;
          acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[x][i][0], Bh[x], acc[x][i][j], 0, 0, 0);
          acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[x][i][0], Bl[x], acc[x][i][j], 0, 0, 0);
          acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[x][i][1], Bh[x], acc[x][i][j], 0, 0, 0);
        }
    }
  };

  // K loop, one step per chunk pair k, one barrier per step.  Per step each wave issues the
  // filters of pair k + 1 (8 loads, into the other register set) and the raw input of pair k + 2
  // (4 LDS-DMA pieces, ring slot (k + 2) % 3), then transforms and multiplies pair k.  Counted
  // waits (loads past the last pair repeat it, so the counts are the same on every step):
  //   before the MFMAs: A(k) landed       -- younger: raw(k+1) 4, A(k+1) 8, raw(k+2) 4 -> vmcnt(16)
  //   before the barrier: raw(k+1) landed -- younger: A(k+1) 8, raw(k+2) 4           -> vmcnt(12)
  f16x8 AS[2][2][2][2];   // two register sets [set][xi][i][hi|lo]
  load_a(AS[0], 0);
  dma(0, 0);
  dma(min(1, a.pairs - 1), 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");       // raw(0) landed (raw(1) may not)
  __syncthreads();                                       // (and the epilogue constants are staged)
  __builtin_amdgcn_sched_barrier(0);
  auto step = [&](int k, f16x8 (&A)[2][2][2], f16x8 (&An)[2][2][2]) __attribute__((always_inline)) {
    load_a(An, min(k + 1, a.pairs - 1));
    dma(min(k + 2, a.pairs - 1), (k + 2) % 3);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((ABL & 4) == 0)
      asm volatile("s_waitcnt vmcnt(16)"
                   : "+v"(A[0][0][0]), "+v"(A[0][0][1]), "+v"(A[0][1][0]), "+v"(A[0][1][1]), "+v"(A[1][0][0]),
                     "+v"(A[1][0][1]), "+v"(A[1][1][0]), "+v"(A[1][1][1])
                   :
                   : "memory");
    compute(A, k % 3);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int k = 0; k < a.pairs; k += 2) {
    step(k, AS[0], AS[1]);
    if (k + 1 < a.pairs) step(k + 1, AS[1], AS[0]);
  }
  // every filter register the asm loads wrote stays allocated until the loads have landed (the
  // last step's loads are never used: without this their registers could be reused while in flight)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)"
               : "+v"(AS[0][0][0][0]), "+v"(AS[0][0][0][1]), "+v"(AS[0][0][1][0]), "+v"(AS[0][0][1][1]),
                 "+v"(AS[0][1][0][0]), "+v"(AS[0][1][0][1]), "+v"(AS[0][1][1][0]), "+v"(AS[0][1][1][1]),
                 "+v"(AS[1][0][0][0]), "+v"(AS[1][0][0][1]), "+v"(AS[1][0][1][0]), "+v"(AS[1][0][1][1]),
                 "+v"(AS[1][1][0][0]), "+v"(AS[1][1][0][1]), "+v"(AS[1][1][1][0]), "+v"(AS[1][1][1][1])
               :
               : "memory");
  __syncthreads();

  bool bad = false;
  if constexpr ((ABL & 16) != 0) {
    // keep the accumulators live: one value per lane
    float sum = 0.f;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) sum += acc[x][i][j][r];
    if (sum == 1.2345f || bad) atomicOr(a.range_flag, 1);
    return;
  }
  // epilogue: M tiles through LDS, per round i (32 channels) [xi][j][q][h][32] x f32x4 (128 KB);
  // thread (j, q, h, tile) sums its 4 channels' 16 values in a fixed order into the 2x2 outputs
  f32x4* xm = smem;
  const float* eb = (const float*)(smem + 8192);
  const int Wo = a.W + 2 * a.out_pad;
  float* out_f = a.out + (size_t)n * a.out_fs;
  const int rn = tid & 31, rh = (tid >> 5) & 1, rq = (tid >> 6) & 3, rj = tid >> 8;
  const int rs = s0 + 32 * rj + rn, rband = rs / BW, ru = rs - rband * BW, rtx = ru >> 1, rty = 2 * rband + (ru & 1);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          xm[((((2 * w + x) * 2 + j) * 4 + q) * 2 + h) * 32 + l32] =
              f32x4{acc[x][i][j][4 * q], acc[x][i][j][4 * q + 1], acc[x][i][j][4 * q + 2], acc[x][i][j][4 * q + 3]};
    __syncthreads();
    {
      const f32x4* mp = xm + ((rj * 4 + rq) * 2 + rh) * 32 + rn;   // + xi * 8 KiB (512 units)
      // Y = A^T M A: rows R0[c] = M0c + M1c + M2c, R1[c] = M1c - M2c - M3c; then the columns
      f32x4 R0[4], R1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f32x4 m0 = mp[(0 + c) * 512], m1 = mp[(4 + c) * 512], m2 = mp[(8 + c) * 512], m3 = mp[(12 + c) * 512];
        R0[c] = (m0 + m1) + m2;
        R1[c] = (m1 - m2) - m3;
      }
      f32x4 Y[2][2];
      Y[0][0] = (R0[0] + R0[1]) + R0[2];
      Y[0][1] = (R0[1] - R0[2]) - R0[3];
      Y[1][0] = (R1[0] + R1[1]) + R1[2];
      Y[1][1] = (R1[1] - R1[2]) - R1[3];
      const int cl = i * 32 + 8 * rq + 4 * rh, co = co_b * 64 + cl;
      const f32x4 bv = *(const f32x4*)(eb + cl);
      const f32x4 sl = *(const f32x4*)(eb + 64 + cl);
      if (rty < a.TH) {
        float* oc = out_f + (size_t)(co >> 3) * a.out_chs + (co & 7);
#pragma unroll
        for (int yy = 0; yy < 2; ++yy)
#pragma unroll
          for (int xx = 0; xx < 2; ++xx) {
            const int y = 2 * rty + yy, x = 2 * rtx + xx;
            if (y >= a.H || x >= a.W) continue;
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = Y[yy][xx][e] * a.wscale_inv + bv[e];
            if (a.act == ACT_RELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
            } else if (a.act == ACT_PRELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * sl[e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) bad |= !(__builtin_fabsf(v[e]) < 65504.f);
            *(f32x4*)(oc + (size_t)((y + a.out_pad) * Wo + x + a.out_pad) * 8) = v;
          }
      }
    }
    __syncthreads();
  }
  if (bad) atomicOr(a.range_flag, 1);
}

int g_wino_blocks(const ConvLaunch& c, int* bpf) {
  const int TH = (c.H + 1) / 2, TW = (c.W + 1) / 2, nbands = (TH + 1) / 2;
  *bpf = (nbands * 2 * TW + 63) / 64;
  return c.n * *bpf * (c.cout / 64);
}

}  // namespace

bool wino_f16_fits(const ConvLaunch& c) {
  return c.ks == 3 && c.in_pad >= 1 && c.cout % 64 == 0 && c.cout > 0 && !c.hpool && !c.vin && !c.fold &&
         c.cout7 == 0 && (c.W + 1) / 2 >= 32 && (long long)c.H * c.W > 1024 &&
         !((c.in_cs | c.in_coff | c.out_cs | c.out_coff) & 7) && (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8 < (1ll << 30);
}

hipError_t launch_wino_f16(const ConvLaunch& c, hipStream_t s) {
  if (!wino_f16_fits(c)) { set_error("wino_f16: launch not eligible"); return hipErrorInvalidValue; }
  if (!c.wx3 || !c.range_flag) { set_error("wino_f16: split filters / range flag missing"); return hipErrorInvalidValue; }
  W2Args a{};
  a.in_chs = (long long)(c.H + 2 * c.in_pad) * (c.W + 2 * c.in_pad) * 8;
  a.out_chs = (long long)(c.H + 2 * c.out_pad) * (c.W + 2 * c.out_pad) * 8;
  a.in_fs = a.in_chs * (c.in_cs / 8);
  a.out_fs = a.out_chs * (c.out_cs / 8);
  a.in = c.in + (c.in_coff / 8) * a.in_chs;
  a.out = c.out + (c.out_coff / 8) * a.out_chs;
  a.upk = (const f16x8*)c.wx3;
  a.bias = c.bias;
  a.slope = c.slope;
  a.range_flag = c.range_flag;
  a.wscale_inv = c.wscale_inv;
  a.in_pad = c.in_pad;
  a.out_pad = c.out_pad;
  a.H = c.H;
  a.W = c.W;
  a.TH = (c.H + 1) / 2;
  a.TW = (c.W + 1) / 2;
  a.pairs = (c.cin_chunks + 1) / 2;
  a.cin_chunks = c.cin_chunks;
  a.co_blocks = c.cout / 64;
  a.act = c.act;
  const long long nb = g_wino_blocks(c, &a.bpf);
  if (nb <= 0 || nb > 0x7fffffff) { set_error("wino_f16: bad grid"); return hipErrorInvalidValue; }
  a.nblocks = (int)nb;
#ifdef ISLPOSE_DEV
  const int abl = getenv("ISLPOSE_W2_ABL") ? atoi(getenv("ISLPOSE_W2_ABL")) : 0;
  switch (abl) {
#define W2ABL(k) case k: hipLaunchKernelGGL(wino_f16<k>, dim3(a.nblocks), dim3(512), 0, s, a); return hipGetLastError();
    W2ABL(1) W2ABL(2) W2ABL(3) W2ABL(4) W2ABL(6) W2ABL(8) W2ABL(12) W2ABL(14) W2ABL(16) W2ABL(31)
#undef W2ABL
    default: break;
  }
#endif
  hipLaunchKernelGGL(wino_f16<0>, dim3(a.nblocks), dim3(512), 0, s, a);
  return hipGetLastError();
}

double wino_f16_mfma_flops(const ConvLaunch& c) {
  int bpf = 0;
  const double nb = g_wino_blocks(c, &bpf);
  return nb * 16.0 * 64 * 64 * 16.0 * ((c.cin_chunks + 1) / 2) * 2 * 3;
}

}  // namespace isl
