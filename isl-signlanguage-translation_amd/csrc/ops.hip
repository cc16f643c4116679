// Byte-moving kernels around the convolutions: 2x2 max-pool, NCHW <-> chunked
// padded packing, and the frame pre-processing of Body/Hand.__call__.
#include <cstring>

#include "internal.h"

namespace isl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// nn.MaxPool2d(2, 2, 0) (model.py:30-31): floor mode, 4 channels per thread;
// thread order (frame, chunk, y, x, half) so a wave reads and writes contiguous bytes.
// 2x2 / stride 2 max-pool (nn.MaxPool2d(2, 2), model.py:33) on chunked buffers.
// Grid: x = pixel halves of one output plane (32-bit index math), y = (frame, chunk)
// plane.  A lane pair covers one output pixel's 8 channels (16 B each), so a
// wave reads two 1 KiB input row runs and writes one 1 KiB output run.
__global__ void maxpool2_kernel(const float* __restrict__ in, int ip, int iH, int iW, float* __restrict__ out,
                                int op, int oH, int oW, int chunks, int in_chunks, int out_chunks) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= oH * oW * 2) return;
  const int plane = blockIdx.y, f = plane / chunks, k = plane - f * chunks;
  const int half = idx & 1, px = idx >> 1;
  const int y = px / oW, x = px - y * oW;
  const int iWp = iW + 2 * ip, oWp = oW + 2 * op;
  const size_t ich = (size_t)(iH + 2 * ip) * iWp * 8, och = (size_t)(oH + 2 * op) * oWp * 8;
  const float* p = in + ((size_t)f * in_chunks + k) * ich + (size_t)((2 * y + ip) * iWp + 2 * x + ip) * 8 + 4 * half;
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 8);
  const f32x4 c = *(const f32x4*)(p + (size_t)iWp * 8), d = *(const f32x4*)(p + (size_t)iWp * 8 + 8);
  f32x4 m;
#pragma unroll
  for (int e = 0; e < 4; ++e) m[e] = fmaxf(fmaxf(a[e], b[e]), fmaxf(c[e], d[e]));
  *(f32x4*)(out + ((size_t)f * out_chunks + k) * och + (size_t)((y + op) * oWp + x + op) * 8 + 4 * half) = m;
}

// Range-guard bookkeeping of isl_net_check_async: a set flag adds one to the net's trip
// counter (read by isl_net_range_info) before the flag is copied out and reset.
__global__ void range_count_kernel(const int* __restrict__ flag, unsigned long long* __restrict__ trips) {
  if (threadIdx.x == 0 && *flag) *trips += 1ull;
}

hipError_t launch_range_count(const int* flag, unsigned long long* trips, hipStream_t s) {
  hipLaunchKernelGGL(range_count_kernel, dim3(1), dim3(64), 0, s, flag, trips);
  return hipGetLastError();
}

hipError_t launch_maxpool2(const Act& in, const Act& out, int C, hipStream_t s) {
  const int chunks = (C + 7) / 8;
  const long long per_plane = (long long)out.H * out.W * 2;
  if (per_plane > 0x7fffffffLL || (long long)out.n * chunks > 65535) {
    set_error("maxpool2: plane too large");
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)((per_plane + 255) / 256), out.n * chunks), dim3(256), 0, s,
                     in.base, in.pad, in.H, in.W, out.base, out.pad, out.H, out.W, chunks, in.cs / 8, out.cs / 8);
  return hipGetLastError();
}

// Second half of a fused 2x2 max-pool: the producing conv's epilogue already took the
// max of each horizontal pixel pair (ConvLaunch::hpool) into an unpadded
// [n][chunk][H][W/2][8] buffer; here each output pixel is the max of its two rows
// (floor mode: an odd last row is dropped, as MaxPool2d(2, 2) does).  Reads half the
// bytes maxpool2_kernel reads, and the conv wrote half the bytes.
__global__ void vpool2_kernel(const float* __restrict__ in, int iH, int iW2, float* __restrict__ out, int op,
                              int oH, int oW, int chunks, int in_chunks, int out_chunks) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= oH * oW * 2) return;
  const int plane = blockIdx.y, f = plane / chunks, k = plane - f * chunks;
  const int half = idx & 1, px = idx >> 1;
  const int y = px / oW, x = px - y * oW;
  const int oWp = oW + 2 * op;
  const size_t ich = (size_t)iH * iW2 * 8, och = (size_t)(oH + 2 * op) * oWp * 8;
  const float* p = in + ((size_t)f * in_chunks + k) * ich + (size_t)(2 * y * iW2 + x) * 8 + 4 * half;
  const f32x4 a = *(const f32x4*)p, c = *(const f32x4*)(p + (size_t)iW2 * 8);
  f32x4 m;
#pragma unroll
  for (int e = 0; e < 4; ++e) m[e] = fmaxf(a[e], c[e]);
  *(f32x4*)(out + ((size_t)f * out_chunks + k) * och + (size_t)((y + op) * oWp + x + op) * 8 + 4 * half) = m;
}

hipError_t launch_vpool2(const Act& in, const Act& out, int C, hipStream_t s) {
  const int chunks = (C + 7) / 8;
  const long long per_plane = (long long)out.H * out.W * 2;
  if (per_plane > 0x7fffffffLL || (long long)out.n * chunks > 65535 || in.pad != 0 || out.W != in.W ||
      out.H != in.H / 2) {
    set_error("vpool2: bad geometry");
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(vpool2_kernel, dim3((unsigned)((per_plane + 255) / 256), out.n * chunks), dim3(256), 0, s,
                     in.base, in.H, in.W, out.base, out.pad, out.H, out.W, chunks, in.cs / 8, out.cs / 8);
  return hipGetLastError();
}

// NCHW float (module seam input) -> chunked padded buffer, channels >= C zero-filled.
__global__ void pack_nchw_kernel(const float* __restrict__ x, int n, int C, int h, int w,
                                 float* __restrict__ out, int op, int ocs) {
  const long long total = (long long)n * h * w;
  const size_t chs = (size_t)(h + 2 * op) * (w + 2 * op) * 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    const int yy = (int)((i / w) % h);
    const int f = (int)(i / ((long long)w * h));
    float* o = out + (size_t)f * (ocs / 8) * chs + ((size_t)(yy + op) * (w + 2 * op) + xx + op) * 8;
    for (int c = 0; c < ocs; ++c)
      o[(size_t)(c >> 3) * chs + (c & 7)] = c < C ? x[(((size_t)f * C + c) * h + yy) * w + xx] : 0.f;
  }
}

hipError_t launch_pack_nchw(const float* x, int n, int C, int h, int w, const Act& out, hipStream_t s) {
  const long long total = (long long)n * h * w;
  const int grid = (int)std::min<long long>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(pack_nchw_kernel, dim3(grid), dim3(256), 0, s, x, n, C, h, w, out.base, out.pad, out.cs);
  return hipGetLastError();
}

// chunked padded slice [coff, coff+C) -> NCHW float (module seam output).
__global__ void unpack_nchw_kernel(const float* __restrict__ in, int ip, int ics, int coff, int n, int C,
                                   int h, int w, float* __restrict__ y) {
  const long long total = (long long)n * C * h * w;
  const size_t chs = (size_t)(h + 2 * ip) * (w + 2 * ip) * 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    long long r = i / w;
    const int yy = (int)(r % h); r /= h;
    const int c = (int)(r % C) + coff;
    const int f = (int)(r / C);
    y[i] = in[((size_t)f * (ics / 8) + (c >> 3)) * chs + ((size_t)(yy + ip) * (w + 2 * ip) + xx + ip) * 8 + (c & 7)];
  }
}

hipError_t launch_unpack_nchw(const Act& in, int coff, int C, float* y, hipStream_t s) {
  const long long total = (long long)in.n * C * in.H * in.W;
  const int grid = (int)std::min<long long>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(unpack_nchw_kernel, dim3(grid), dim3(256), 0, s, in.base, in.pad, in.cs, coff, in.n, C,
                     in.H, in.W, y);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Frame pre-processing (body.py:53-56, hand.py:37-40):
//   cv2.resize(uint8 BGR, fx=fy=scale, INTER_CUBIC) -> padRightDownCorner(8, 128)
//   -> float32(img)/256 - 0.5, written as chunk 0 of the padded input buffer
//   (3 real + 5 zero channels).
// The uint8 cubic follows OpenCV's generic path (see oracle/cv_resize.py):
// 11-bit fixed-point coefficients, int horizontal sums, and a vertical pass that
// is float (beta/2^22, round-half-even) for the SIMD body of each output row and
// fixed point ((sum + 2^21) >> 22) for its scalar tail.
// ---------------------------------------------------------------------------

__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  const float A = -0.75f;
  const float tp1 = t + 1.f;
  c[0] = ((A * tp1 - 5.f * A) * tp1 + 8.f * A) * tp1 - 4.f * A;
  c[1] = ((A + 2.f) * t - (A + 3.f)) * t * t + 1.f;
  const float u = 1.f - t;
  c[2] = ((A + 2.f) * u - (A + 3.f)) * u * u + 1.f;
  c[3] = 1.f - c[0] - c[1] - c[2];
}

__device__ __forceinline__ void axis_tap(int d, double scale, int n, int idx[4], float c[4]) {
  float f = (float)((d + 0.5) * scale - 0.5);
  const int s = (int)floorf(f);
  f -= (float)s;
  cubic_coeffs(f, c);
#pragma unroll
  for (int k = 0; k < 4; ++k) idx[k] = min(max(s + k - 1, 0), n - 1);
}

// One image of a preprocess batch: a frame, or a crop of one (Hand.__call__ runs
// on oriImg[y:y+w, x:x+w] views, demo.py:36 / ISL_Model_parameter.py:56).
struct PreSrc {
  long long off;       // byte offset of the image's (0, 0) pixel in the frame array
  int sh, sw;          // image size
  int rh, rw;          // resized size (cvRound(s * fx)); the rest of the net input is pad 128
  double scale;        // source pixels per output pixel (1 / fx)
};

// `tab` (device) describes image f = blockIdx.y; `row` = bytes per source row (frame W * 3).
__global__ void preprocess_kernel(const uint8_t* __restrict__ frames, const PreSrc* __restrict__ tab, long long row,
                                  float* __restrict__ out, int op, int ocs, int ph, int pw) {
  const int f = blockIdx.y;
  const PreSrc t = tab[f];
  const int rowlen = t.rw * 3;
  const int body = rowlen - rowlen % 8;
  const bool identity = t.rh == t.sh && t.rw == t.sw;
  const uint8_t* img = frames + t.off;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ph * pw; i += gridDim.x * blockDim.x) {
    const int y = i / pw, x = i - y * pw;
    float v[3];
    if (y >= t.rh || x >= t.rw) {
      v[0] = v[1] = v[2] = 128.f / 256.f - 0.5f;
    } else if (identity) {
      const uint8_t* p = img + (size_t)y * row + (size_t)x * 3;
      for (int c = 0; c < 3; ++c) v[c] = (float)p[c] / 256.f - 0.5f;
    } else {
      int xi[4], yi[4];
      float xc[4], yc[4];
      axis_tap(x, t.scale, t.sw, xi, xc);
      axis_tap(y, t.scale, t.sh, yi, yc);
      int ia[4], ib[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ia[k] = (int)rintf(xc[k] * 2048.f);
        ib[k] = (int)rintf(yc[k] * 2048.f);
      }
      for (int c = 0; c < 3; ++c) {
        int hz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint8_t* r = img + (size_t)yi[k] * row + c;
          hz[k] = r[xi[0] * 3] * ia[0] + r[xi[1] * 3] * ia[1] + r[xi[2] * 3] * ia[2] + r[xi[3] * 3] * ia[3];
        }
        int r;
        if (x * 3 + c < body) {
          const float sc = 1.f / (2048.f * 2048.f);
          const float b0 = (float)ib[0] * sc, b1 = (float)ib[1] * sc, b2 = (float)ib[2] * sc, b3 = (float)ib[3] * sc;
          const float s = (float)hz[0] * b0 + ((float)hz[1] * b1 + ((float)hz[2] * b2 + (float)hz[3] * b3));
          r = (int)rintf(s);
        } else {
          const long long acc = (long long)hz[0] * ib[0] + (long long)hz[1] * ib[1] + (long long)hz[2] * ib[2] +
                                (long long)hz[3] * ib[3];
          r = (int)((acc + (1 << 21)) >> 22);
        }
        r = min(max(r, 0), 255);
        v[c] = (float)r / 256.f - 0.5f;
      }
    }
    // chunk 0 of the (chunked) input buffer: 3 real + 5 zero channels
    float* o = out + (size_t)f * (ocs / 8) * (ph + 2 * op) * (pw + 2 * op) * 8 +
               ((size_t)(y + op) * (pw + 2 * op) + x + op) * 8;
    *(f32x4*)o = f32x4{v[0], v[1], v[2], 0.f};
    *(f32x4*)(o + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// `tab` is a device array of n PreSrc entries (one per image of the batch).
hipError_t launch_preprocess_tab(const uint8_t* frames, long long row_bytes, const void* tab, int n, const Act& out,
                                 hipStream_t s) {
  if (n > 65535) { set_error("preprocess: batch too large"); return hipErrorInvalidValue; }
  const int blocks = (int)std::min<long long>(((long long)out.H * out.W + 255) / 256, 1024);
  hipLaunchKernelGGL(preprocess_kernel, dim3(blocks, n), dim3(256), 0, s, frames, (const PreSrc*)tab, row_bytes,
                     out.base, out.pad, out.cs, out.H, out.W);
  return hipGetLastError();
}

size_t preprocess_entry_bytes() { return sizeof(PreSrc); }

void preprocess_entry(void* dst, long long off, int sh, int sw, int rh, int rw, double scale) {
  PreSrc t;
  t.off = off; t.sh = sh; t.sw = sw; t.rh = rh; t.rw = rw; t.scale = scale;
  memcpy(dst, &t, sizeof(t));
}

}  // namespace isl
