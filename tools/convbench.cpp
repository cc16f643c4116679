// Conv-kernel microbenchmark (development tool, not shipped): times one conv
// layer shape on random data with every algorithm, interleaved in one process.
//   build: make convbench          run: tools/convbench ks cin cout H W n iters
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "internal.h"

using namespace isl;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));      \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

template <class T>
static T* dev_random(size_t n, float lo, float hi, unsigned seed) {
  std::vector<T> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> d(lo, hi);
  for (auto& v : h) v = (T)d(g);
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  if (argc < 8) {
    fprintf(stderr, "usage: convbench ks cin cout H W n iters [algos=x3,direct,wino] [rounds=3]\n");
    return 2;
  }
  const int ks = atoi(argv[1]), cin = atoi(argv[2]), cout = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]),
            n = atoi(argv[6]), iters = atoi(argv[7]);
  const std::string algos = argc > 8 ? argv[8] : "x3,direct,wino";
  const int rounds = argc > 9 ? atoi(argv[9]) : 3;
  // CONVBENCH_CS=c: input and output are channel slices of c-channel buffers (the net's
  // zero-copy concat: a stage conv reads [0, cin) and writes [cout, 2 cout) of 384-channel
  // buffers)
  const int cs_wide = getenv("CONVBENCH_CS") ? atoi(getenv("CONVBENCH_CS")) : 0;
  const int cs_in = std::max(cs_wide, (cin + 7) / 8 * 8), cs_out = std::max(cs_wide, (cout + 7) / 8 * 8);
  const int pin = std::max(1, ks / 2), pout = 1;
  Act in, out;
  in.n = out.n = n; in.H = out.H = H; in.W = out.W = W;
  in.pad = pin; in.cs = cs_in; out.pad = pout; out.cs = cs_out;
  in.base = dev_random<float>(in.bytes() / 4, -1.f, 1.f, 1);
  CK(hipMalloc(&out.base, out.bytes()));
  // env CONVBENCH_BCO overrides the output-channel tile (timing of other tile families)
  const int bco = getenv("CONVBENCH_BCO") ? atoi(getenv("CONVBENCH_BCO")) : conv_bco_for(cout);
  const int chunks = (cin + 7) / 8, pairs = (chunks + 1) / 2, co_tiles = (cout + bco - 1) / bco;
  float* wd = dev_random<float>((size_t)co_tiles * chunks * ks * ks * 2 * bco * 4, -0.05f, 0.05f, 2);
  _Float16* wx = dev_random<_Float16>((size_t)co_tiles * pairs * ks * ks * 4 * bco * 8, -8192.f, 8192.f, 3);
  const int wb = wino_bco_for(cout);
  float* wu = wb ? dev_random<float>((size_t)(cout / wb) * chunks * 16 * 2 * wb * 4, -0.05f, 0.05f, 4) : nullptr;
  const int wxt = (cout + 63) / 64;
  _Float16* wux = dev_random<_Float16>((size_t)wxt * pairs * 16 * 4 * 64 * 8, -8192.f, 8192.f, 7);
  // split-fp16 Winograd filters of wino_f16 (w2): [cout/64][pair][16][2][2][2][32][8]
  _Float16* ww = cout % 64 == 0 ? dev_random<_Float16>((size_t)(cout / 64) * pairs * 16 * 8 * 32 * 8, -8192.f, 8192.f, 9)
                                : nullptr;
  _Float16* f7w = dev_random<_Float16>((size_t)2 * ((cout + 15) / 16) * 2 * 64 * 8, -8192.f, 8192.f, 8);
  float* bias = dev_random<float>(co_tiles * 256 + 256, -0.05f, 0.05f, 5);
  float* slope = dev_random<float>(co_tiles * 256 + 256, 0.05f, 0.25f, 6);
  int* flag;
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(flag, 0, 4));
  ConvLaunch L;
  L.in = in.base; L.in_pad = pin; L.in_cs = cs_in; L.in_coff = 0;
  L.out = out.base; L.out_pad = pout; L.out_cs = cs_out; L.out_coff = cs_wide >= 2 * cout ? (cout + 7) / 8 * 8 : 0;
  L.bias = bias; L.slope = slope; L.n = n; L.H = H; L.W = W; L.ks = ks; L.cin_chunks = chunks; L.cout = cout;
  L.act = ACT_PRELU; L.wx3 = wx; L.wscale_inv = 1.f / 16384.f; L.range_flag = flag;
  // CONVBENCH_SPLIT=1|2: the net's K-range mode (canonical ranges / latency split), with a workspace
  if (getenv("CONVBENCH_SPLIT")) {
    L.allow_split = atoi(getenv("CONVBENCH_SPLIT"));
    L.bco = bco;
    L.ws_floats = x3_splitk_ws_floats(L);
    if (L.ws_floats) CK(hipMalloc(&L.ws, L.ws_floats * sizeof(float)));
  }
  // ISLPOSE_X3_UNION=4: s_memtime stamps of block 0 (16 waves x K steps x 4 points)
  const int T = pairs * ks;
  unsigned long long* dbg = nullptr;
  if (getenv("ISLPOSE_X3_UNION") && atoi(getenv("ISLPOSE_X3_UNION")) == 4) {
    CK(hipMalloc(&dbg, ((size_t)16 * T * 4 + 4) * 8));
    CK(hipMemset(dbg, 0, ((size_t)16 * T * 4 + 4) * 8));
    L.dbg = dbg;
  }
  // CONVBENCH_WRSTAMP=1: phase stamps of the wave-range kernel (conv_x3_wr, wave 0 of every block)
  const bool wrstamp = getenv("CONVBENCH_WRSTAMP") && atoi(getenv("CONVBENCH_WRSTAMP"));
  const size_t wr_blocks = 1 << 16;
  if (wrstamp) {
    CK(hipMalloc(&dbg, wr_blocks * 8 * 8));
    CK(hipMemset(dbg, 0, wr_blocks * 8 * 8));
    L.dbg = dbg;
  }
  const double flops = 2.0 * cout * cin * ks * ks * (double)H * W * n;
  // the polluter of CONVBENCH_POLLUTE: a 1x1 layer on the same buffers (cin chunks of this
  // shape, 32 output channels), default variant
  const bool pollute = getenv("CONVBENCH_POLLUTE") && atoi(getenv("CONVBENCH_POLLUTE"));
  ConvLaunch PL = L;
  PL.ks = 1; PL.cout = 32; PL.bco = 32; PL.ws = nullptr; PL.ws_floats = 0; PL.allow_split = 0;
  void* flush = nullptr;
  const size_t flush_bytes = (size_t)1 << 30;
  if (getenv("CONVBENCH_FLUSH") && atoi(getenv("CONVBENCH_FLUSH"))) CK(hipMalloc(&flush, flush_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("conv k%d %d->%d %dx%d n=%d: %.2f GFLOP (direct count)\n", ks, cin, cout, H, W, n, flops / 1e9);
  for (int r = 0; r < rounds; ++r) {
    size_t pos = 0;
    while (pos < algos.size()) {
      size_t e = algos.find(',', pos);
      if (e == std::string::npos) e = algos.size();
      const std::string a = algos.substr(pos, e - pos);
      pos = e + 1;
      ConvLaunch c = L;
      auto launch = [&]() -> hipError_t {
        // x3m: the row union on 16x16x32 MFMAs (ISLPOSE_X3_M16=1, read per launch); x3: off
        // x3h: small grids on two 64-channel blocks per 128-channel tile (ISLPOSE_X3_HALFCO=1)
        // x3p: small grids with two chunk pairs per K step (ISLPOSE_X3_PPS2=1)
        // x3d: small grids with inputs and weights two K steps ahead (ISLPOSE_X3_DEEP=1)
        if (a == "x3" || a == "x3m" || a == "x3h" || a == "x3p" || a == "x3d") {
          setenv("ISLPOSE_X3_DEEP", a == "x3d" ? "1" : "0", 1);
          setenv("ISLPOSE_X3_M16", a == "x3m" ? "1" : "0", 1);
          setenv("ISLPOSE_X3_HALFCO", a == "x3h" ? "1" : "0", 1);
          setenv("ISLPOSE_X3_PPS2", a == "x3p" ? "1" : "0", 1);
          c.bco = bco; c.wpk = wd;
          return launch_conv_x3(c, 0);
        }
        // x3f: the fused 1x1 pair (cout = Mconv6 channels; CONVBENCH_F7 Mconv7 outputs, default 52)
        if (a == "x3f" && ks == 1) {
          c.cout7 = getenv("CONVBENCH_F7") ? atoi(getenv("CONVBENCH_F7")) : 52;
          c.wx3f7 = f7w; c.bias7 = bias; c.slope7 = slope; c.act7 = ACT_PRELU; c.wscale7_inv = 1.f / 16384.f;
          c.out_cs = 64; c.bco = cout; c.wpk = wd;
          return launch_conv_x3(c, 0);
        }
        if (a == "direct") { c.bco = bco; c.wpk = wd; return launch_conv(c, 0); }
        if (a == "wino" && wb && ks == 3) { c.bco = wb; c.wpk = wu; return launch_wino(c, 0); }
        if (a == "wx3" && ks == 3) { c.wx3 = wux; return launch_wino_x3(c, 0); }
        // w2: the split-fp16 Winograd kernel wino_f16 (ISLPOSE_W2_ABL: its timing ablations)
        if (a == "w2" && ww && wino_f16_fits(c)) { c.wx3 = ww; return launch_wino_f16(c, 0); }
        return hipErrorNotSupported;
      };
      if (launch() != hipSuccess) continue;
      for (int i = 0; i < 2; ++i) CK(launch());
      float ms = 0.f;
      if (flush || pollute) {
        // CONVBENCH_FLUSH=1: caches cold before every launch (a 1 GiB memset evicts L2 and the
        // Infinity Cache), each launch timed alone -- the net's first touch of a layer's weights.
        // CONVBENCH_POLLUTE=1: a launch of the conv_x3 variant of another shape (a 1x1 layer)
        // before every timed launch, as in the net, where kernels of other shapes alternate
        for (int i = 0; i < iters; ++i) {
          if (flush) CK(hipMemsetAsync(flush, i & 0xff, flush_bytes, 0));
          if (pollute) CK(launch_conv_x3(PL, 0));
          CK(hipEventRecord(e0, 0));
          CK(launch());
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float m1;
          CK(hipEventElapsedTime(&m1, e0, e1));
          ms += m1;
        }
      } else {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) CK(launch());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double us = ms * 1e3 / iters;
      const double fac = (a == "x3" || a == "x3f" || a == "x3m" || a == "x3h" || a == "x3p" || a == "x3d") ? 3.0 : (a == "wx3" || a == "w2") ? 3.0 * 16 / 36 : a == "wino" ? 16.0 / 36 : 1.0;
      printf("  round %d %-7s %9.1f us  fp32-equiv %7.1f TF  alg-MFMA %7.1f TF\n", r, a.c_str(), us,
             flops / us / 1e6, fac * flops / us / 1e6);
    }
  }
  if (dbg && wrstamp) {
    std::vector<unsigned long long> h(wr_blocks * 8);
    CK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
    double ph[4] = {0, 0, 0, 0}, t0min = 1e300, t0max = 0, t4max = 0, clk = 0;
    int nb = 0;
    for (size_t b = 0; b < wr_blocks && h[b * 8]; ++b, ++nb) {
      for (int k = 0; k < 4; ++k) ph[k] += (double)h[b * 8 + k + 1] - (double)h[b * 8 + k];
      t0min = std::min(t0min, (double)h[b * 8]);
      t0max = std::max(t0max, (double)h[b * 8]);
      t4max = std::max(t4max, (double)h[b * 8 + 4]);
      const double dr = (double)h[b * 8 + 7] - (double)h[b * 8 + 6];
      if (dr > 0) clk += ((double)h[b * 8 + 4] - (double)h[b * 8]) / dr * 0.1;
    }
    if (nb)
      printf("  wr stamps (%d blocks, cycles, mean): first operands %.0f, K loop %.0f, combine %.0f, epilogue %.0f; "
             "block starts spread %.0f, first start to last end %.0f; clock %.2f GHz\n", nb, ph[0] / nb, ph[1] / nb,
             ph[2] / nb, ph[3] / nb, t0max - t0min, t4max - t0min, clk / nb);
  } else if (dbg) {
    // per step: issue (0->1), compute (1->2), store (2->3), barrier (3 -> next 0), for
    // the earliest and latest wave, averaged over the steps of the last launch
    std::vector<unsigned long long> h((size_t)16 * T * 4 + 4);
    CK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
    auto at = [&](int w, int t, int k) { return (double)h[((size_t)w * T + t) * 4 + k]; };
    double ph[4] = {0, 0, 0, 0}, step = 0;
    int nst = 0;
    for (int t = 1; t + 1 < T; ++t, ++nst) {
      double mn0 = 1e300, mx3 = 0;
      for (int w = 0; w < 16; ++w) {
        ph[0] += (at(w, t, 1) - at(w, t, 0)) / 16;
        ph[1] += (at(w, t, 2) - at(w, t, 1)) / 16;
        ph[2] += (at(w, t, 3) - at(w, t, 2)) / 16;
        ph[3] += (at(w, t + 1, 0) - at(w, t, 3)) / 16;
        mn0 = std::min(mn0, at(w, t, 0));
        mx3 = std::max(mx3, at(w, t, 3));
      }
      step += at(0, t + 1, 0) - at(0, t, 0);
    }
    printf("  stamps (cycles per step, mean over waves and %d steps): issue %.0f compute %.0f store %.0f barrier %.0f; "
           "step %.0f\n", nst, ph[0] / nst, ph[1] / nst, ph[2] / nst, ph[3] / nst, step / nst);
    {
      const double* z = nullptr;
      (void)z;
      const double dt = (double)h[(size_t)16 * T * 4 + 2] - (double)h[(size_t)16 * T * 4];
      const double dr = (double)h[(size_t)16 * T * 4 + 3] - (double)h[(size_t)16 * T * 4 + 1];
      if (dr > 0) printf("  in-kernel clock (s_memtime / s_memrealtime x 100 MHz, steps 1..T-1): %.3f GHz\n", dt / dr * 0.1);
    }
    for (int w = 0; w < 16; ++w)
      printf("    wave %2d step 5: compute %.0f store %.0f wait %.0f\n", w, at(w, 5, 2) - at(w, 5, 1),
             at(w, 5, 3) - at(w, 5, 2), at(w, 6, 0) - at(w, 5, 3));
  }
  return 0;
}
