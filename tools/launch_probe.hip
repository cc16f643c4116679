// Dependent-launch cost on one stream: how much of a batch-1 kernel's ~7.5 us
// is the launch itself.  Chains of K launches of
//   empty1    an empty kernel, 1 block of 64 threads
//   empty256  an empty kernel, 256 blocks of 256 threads
//   write2mb  256 blocks writing 2 MB (a 23x41 c128 frame's fp32 output: 0.48 MB x4 ranges)
//   rw2mb     256 blocks reading 8 MB and writing 2 MB (the split-K reduce's traffic at batch 1)
// timed with HIP events, eager and as one captured graph.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void empty_kernel(int) {}

__global__ void write_kernel(float4* __restrict__ out, int n4) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
    out[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ void rw_kernel(const float4* __restrict__ in, float4* __restrict__ out, int n4) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    float4 a = in[i], b = in[i + n4], c = in[i + 2 * n4], d = in[i + 3 * n4];
    out[i] = make_float4(a.x + b.x + c.x + d.x, a.y + b.y + c.y + d.y, a.z + b.z + c.z + d.z,
                         a.w + b.w + c.w + d.w);
  }
}

static void launch(int kind, float4* in, float4* out, int n4, hipStream_t s) {
  switch (kind) {
    case 0: hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, 0); break;
    case 1: hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, 0); break;
    case 2: hipLaunchKernelGGL(write_kernel, dim3(256), dim3(256), 0, s, out, n4); break;
    case 3: hipLaunchKernelGGL(rw_kernel, dim3(256), dim3(256), 0, s, in, out, n4); break;
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 500;
  const int n4 = (2 << 20) / 16;
  float4 *in, *out;
  CK(hipMalloc(&in, (size_t)4 * n4 * sizeof(float4)));
  CK(hipMalloc(&out, (size_t)n4 * sizeof(float4)));
  CK(hipMemset(in, 0, (size_t)4 * n4 * sizeof(float4)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[4] = {"empty1", "empty256", "write2mb", "rw2mb"};
  for (int kind = 0; kind < 4; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      for (int i = 0; i < 50; ++i) launch(kind, in, out, n4, s);
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < K; ++i) launch(kind, in, out, n4, s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      // the same chain as one graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < K; ++i) launch(kind, in, out, n4, s);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float gms = 0;
      CK(hipEventElapsedTime(&gms, e0, e1));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      printf("%-9s eager %6.2f us/launch   graph %6.2f us/launch\n", names[kind], 1e3 * ms / K, 1e3 * gms / K);
    }
  }
  return 0;
}
