// Development microbenchmark (not part of the library): the x3 inner loop -- fragments
// read from LDS by ds_read_b128, 3 fp16 MFMAs per product (hi*hi, hi*lo, lo*hi) into a
// 64co x 64px wave tile -- with v_mfma_f32_32x32x16_f16 (what conv_x3 uses) against
// v_mfma_f32_16x16x32_f16 at the same FLOPs and LDS bytes, on random split operands.
// MI355X_MICROARCH.md (DVFS give-back item 7) measured the 16x16x32 form ~1.12-1.15x
// faster in FLOP/s under DVFS at equal cycles per FLOP.  Prints TFLOP/s and the in-kernel
// clock (s_memtime / s_memrealtime) per shape.
//   build: hipcc -O3 --offload-arch=gfx950 tools/mfma_shape_bench.hip -o tools/mfma_shape_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));        \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int LDS_UNITS = 8192;   // 128 KiB of f16x8
constexpr int NT = 1024;          // 16 waves

// 32x32x16: per iteration (K = 16) per wave 2 A x 2 (hi, lo) + 2 B x 2 reads, 4 tiles x 3 MFMAs
__global__ void __launch_bounds__(NT, 4) loop32(const f16x8* g, float* out, int iters, unsigned long long* clk) {
  __shared__ f16x8 s[LDS_UNITS];
  for (int i = threadIdx.x; i < LDS_UNITS; i += NT) s[i] = g[(blockIdx.x * 131 + i) % (4 * LDS_UNITS)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x16 acc[2][2] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  int off = (wave * 64 + lane) & (LDS_UNITS / 2 - 1);
  for (int it = 0; it < iters; ++it) {
    f16x8 A[2][2], B[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        A[m][hl] = s[(off + m * 32 + hl * 1024) & (LDS_UNITS - 1)];
        B[m][hl] = s[(off + m * 32 + hl * 1024 + 2048 + 7) & (LDS_UNITS - 1)];
      }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][1], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][1], B[n][0], acc[m][n], 0, 0, 0);
      }
    off = (off + 64) & (LDS_UNITS / 2 - 1);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) v += acc[m][n][r];
  out[blockIdx.x * NT + threadIdx.x] = v;
}

// 16x16x32: per iteration (K = 32, so twice the K of loop32: 2 x its FLOPs) per wave
// 4 A x 2 + 4 B x 2 reads, 16 tiles x 3 MFMAs
__global__ void __launch_bounds__(NT, 4) loop16(const f16x8* g, float* out, int iters, unsigned long long* clk) {
  __shared__ f16x8 s[LDS_UNITS];
  for (int i = threadIdx.x; i < LDS_UNITS; i += NT) s[i] = g[(blockIdx.x * 131 + i) % (4 * LDS_UNITS)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 acc[4][4] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  int off = (wave * 64 + lane) & (LDS_UNITS / 2 - 1);
  for (int it = 0; it < iters; ++it) {
    f16x8 A[4][2], B[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        A[m][hl] = s[(off + m * 16 + hl * 1024) & (LDS_UNITS - 1)];
        B[m][hl] = s[(off + m * 16 + hl * 1024 + 2048 + 7) & (LDS_UNITS - 1)];
      }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][0], B[n][1], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][1], B[n][0], acc[m][n], 0, 0, 0);
      }
    off = (off + 64) & (LDS_UNITS / 2 - 1);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += acc[m][n][r];
  out[blockIdx.x * NT + threadIdx.x] = v;
}

// loop32 variants for the power question (is the LDS traffic or the barrier what keeps the
// conv's clock / MFMA issue down?): RD = re-read the fragments from LDS every RD-th
// iteration only (RD = 1 is loop32), BAR = a __syncthreads every 3 iterations (one conv
// step: 36 MFMAs per wave between barriers).
template <int RD, bool BAR>
__global__ void __launch_bounds__(NT, 4) var32(const f16x8* g, float* out, int iters, unsigned long long* clk) {
  __shared__ f16x8 s[LDS_UNITS];
  for (int i = threadIdx.x; i < LDS_UNITS; i += NT) s[i] = g[(blockIdx.x * 131 + i) % (4 * LDS_UNITS)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x16 acc[2][2] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  int off = (wave * 64 + lane) & (LDS_UNITS / 2 - 1);
  f16x8 A[2][2], B[2][2];
  for (int it = 0; it < iters; ++it) {
    if (it % RD == 0) {
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
          A[m][hl] = s[(off + m * 32 + hl * 1024) & (LDS_UNITS - 1)];
          B[m][hl] = s[(off + m * 32 + hl * 1024 + 2048 + 7) & (LDS_UNITS - 1)];
        }
      off = (off + 64) & (LDS_UNITS / 2 - 1);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][1], acc[m][n], 0, 0, 0);
        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][1], B[n][0], acc[m][n], 0, 0, 0);
      }
    if (BAR && it % 3 == 2) __syncthreads();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) v += acc[m][n][r];
  out[blockIdx.x * NT + threadIdx.x] = v;
}

// One 3x3 (pair, ky) step of the conv, both shapes, equal useful FLOPs per iteration:
// 3 taps x 2 chunks x 3 terms = 18 fragment units of K = 8 per output tile.
// step32: per tap A hi/lo x 2, B hi/lo x 2 reads, 4 tiles x 3 MFMAs (36 MFMAs, 24 reads).
// step16: taps 0+1 as 3 full 16x16x32 MFMAs (hi/lo reuse kept), tap 2's 6 units packed
// into 2 MFMAs whose second one is half zero (lanes 32-63 read a zeroed LDS region):
// 16 tiles x 5 MFMAs = 80 (72 useful), 32 reads.
constexpr int ZERO = LDS_UNITS;   // 64 zeroed units after the data
__global__ void __launch_bounds__(NT, 4) step32(const f16x8* g, float* out, int iters, unsigned long long* clk) {
  __shared__ f16x8 s[LDS_UNITS + 64];
  for (int i = threadIdx.x; i < LDS_UNITS; i += NT) s[i] = g[(blockIdx.x * 131 + i) % (4 * LDS_UNITS)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x16 acc[2][2] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  int off = (wave * 64 + lane) & (LDS_UNITS / 2 - 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      f16x8 A[2][2], B[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
          A[m][hl] = s[(off + kx * 256 + m * 32 + hl * 1024) & (LDS_UNITS - 1)];
          B[m][hl] = s[(off + kx * 8 + m * 32 + hl * 1024 + 2048 + 7) & (LDS_UNITS - 1)];
        }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][0], B[n][1], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[m][1], B[n][0], acc[m][n], 0, 0, 0);
        }
    }
    off = (off + 64) & (LDS_UNITS / 2 - 1);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) v += acc[m][n][r];
  out[blockIdx.x * NT + threadIdx.x] = v;
}

__global__ void __launch_bounds__(NT, 4) step16(const f16x8* g, float* out, int iters, unsigned long long* clk) {
  __shared__ f16x8 s[LDS_UNITS + 64];
  for (int i = threadIdx.x; i < LDS_UNITS; i += NT) s[i] = g[(blockIdx.x * 131 + i) % (4 * LDS_UNITS)];
  if (threadIdx.x < 64) s[ZERO + threadIdx.x] = f16x8{};
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 acc[4][4] = {};
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  int off = (wave * 64 + lane) & (LDS_UNITS / 2 - 1);
  const bool upper = lane >= 32;
  for (int it = 0; it < iters; ++it) {
    {  // taps 0 + 1: hh, hl, lh with fragment reuse
      f16x8 A[4][2], B[4][2];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) {
          A[m][hl] = s[(off + m * 16 + hl * 1024) & (LDS_UNITS - 1)];
          B[m][hl] = s[(off + m * 16 + hl * 1024 + 2048 + 7) & (LDS_UNITS - 1)];
        }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][0], B[n][1], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][1], B[n][0], acc[m][n], 0, 0, 0);
        }
    }
    {  // tap 2: [hh c0 c1 | hl c0 c1] and [lh c0 c1 | zero]
      f16x8 A[4][2], B[4][2];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        A[m][0] = s[(off + 512 + m * 16) & (LDS_UNITS - 1)];
        A[m][1] = s[upper ? ZERO + lane : (off + 512 + m * 16 + 1024) & (LDS_UNITS - 1)];
        B[m][0] = s[(off + 8 + m * 16 + 2048 + 7) & (LDS_UNITS - 1)];
        B[m][1] = s[(off + 8 + m * 16 + 3072 + 7) & (LDS_UNITS - 1)];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][0], B[n][0], acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[m][1], B[n][1], acc[m][n], 0, 0, 0);
        }
    }
    off = (off + 64) & (LDS_UNITS / 2 - 1);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  float v = 0.f;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += acc[m][n][r];
  out[blockIdx.x * NT + threadIdx.x] = v;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1024;
  const int iters = argc > 2 ? atoi(argv[2]) : 4000;
  const int rounds = argc > 3 ? atoi(argv[3]) : 4;
  // split-fp16 operands of random fp32 data: hi and lo planes as conv_x3 stages them
  std::vector<_Float16> h((size_t)4 * LDS_UNITS * 8);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> d(-1.f, 1.f);
  for (size_t i = 0; i < h.size(); i += 2) {
    const float x = d(rng) * 8192.f;
    const _Float16 hi = (_Float16)x;
    h[i] = hi;
    h[i + 1] = (_Float16)(x - (float)hi);
  }
  f16x8* g;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&g, h.size() * 2));
  CK(hipMemcpy(g, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)blocks * NT * 4));
  CK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; ++r) {
    for (int k = 0; k < 2; ++k) {
      // equal FLOPs: loop16 does twice the K per iteration, so half the iterations
      const int n_it = k == 0 ? iters : iters / 2;
      CK(hipEventRecord(e0, 0));
      for (int rep = 0; rep < 5; ++rep) {
        if (k == 0) hipLaunchKernelGGL(loop32, dim3(blocks), dim3(NT), 0, 0, g, out, n_it, clk);
        else hipLaunchKernelGGL(loop16, dim3(blocks), dim3(NT), 0, 0, g, out, n_it, clk);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long c[2];
      CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
      // FLOPs per launch: blocks x 16 waves x iters x 4 tiles x 3 x 32x32x16x2
      const double fl = 5.0 * blocks * 16.0 * iters * 4 * 3 * 32768.0;
      printf("round %d %s: %.1f us/launch  %.1f TFLOP/s  in-kernel clock %.3f GHz\n", r,
             k == 0 ? "32x32x16" : "16x16x32", ms * 1e3 / 5, fl / (ms * 1e-3) / 1e12,
             c[1] ? (double)c[0] / c[1] * 0.1 : 0.0);
    }
  }
  // loop32 variants: fragments re-read every iteration / every 16th; a barrier every 3
  if (argc > 4 && argv[4][0] == 'v') {
    for (int r = 0; r < rounds; ++r) {
      for (int k = 0; k < 4; ++k) {
        CK(hipEventRecord(e0, 0));
        for (int rep = 0; rep < 5; ++rep) {
          if (k == 0) hipLaunchKernelGGL((var32<1, false>), dim3(blocks), dim3(NT), 0, 0, g, out, iters, clk);
          else if (k == 1) hipLaunchKernelGGL((var32<16, false>), dim3(blocks), dim3(NT), 0, 0, g, out, iters, clk);
          else if (k == 2) hipLaunchKernelGGL((var32<1, true>), dim3(blocks), dim3(NT), 0, 0, g, out, iters, clk);
          else hipLaunchKernelGGL((var32<16, true>), dim3(blocks), dim3(NT), 0, 0, g, out, iters, clk);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long c[2];
        CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
        const double fl = 5.0 * blocks * 16.0 * iters * 4 * 3 * 32768.0;
        static const char* nm[4] = {"lds every iter", "lds every 16th", "lds + barrier/3", "regs + barrier/3"};
        printf("round %d var32 %-17s: %.1f us/launch  %.1f TFLOP/s  in-kernel clock %.3f GHz\n", r, nm[k],
               ms * 1e3 / 5, fl / (ms * 1e-3) / 1e12, c[1] ? (double)c[0] / c[1] * 0.1 : 0.0);
      }
    }
    return 0;
  }
  // the conv-step pair: useful FLOPs per iteration per wave = 3 taps x 4 tiles x 3 x 32x32x16
  for (int r = 0; r < rounds; ++r) {
    for (int k = 0; k < 2; ++k) {
      const int n_it = iters / 3;
      CK(hipEventRecord(e0, 0));
      for (int rep = 0; rep < 5; ++rep) {
        if (k == 0) hipLaunchKernelGGL(step32, dim3(blocks), dim3(NT), 0, 0, g, out, n_it, clk);
        else hipLaunchKernelGGL(step16, dim3(blocks), dim3(NT), 0, 0, g, out, n_it, clk);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long c[2];
      CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
      const double fl = 5.0 * blocks * 16.0 * n_it * 36 * 32768.0;
      printf("round %d step %s: %.1f us/launch  %.1f useful TFLOP/s  in-kernel clock %.3f GHz\n", r,
             k == 0 ? "32x32x16 (36 MFMA)" : "16x16x32 (80 MFMA, 72 useful)", ms * 1e3 / 5,
             fl / (ms * 1e-3) / 1e12, c[1] ? (double)c[0] / c[1] * 0.1 : 0.0);
    }
  }
  return 0;
}
