// Internal declarations shared by the libislpose translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace isl {

// Activation buffer: float32 in 8-channel chunks ("NC8HW8"), with a zero ring of
// `pad` pixels around every frame, i.e. element (n, y, x, c) lives at
//   base + ((n*(cs/8) + c/8) * (H+2p) + y+p) * (W+2p) * 8 + (x+p) * 8 + c%8.
// A chunk of consecutive pixels is contiguous, so every kernel that walks pixels
// for a K step of 8 channels reads whole cache lines.  Convolutions read/write
// channel slices [coff, coff+C) (coff a multiple of 8) of such buffers, which is
// how every torch.cat of the reference becomes zero-copy.
struct Act {
  float* base = nullptr;
  int n = 0, H = 0, W = 0, pad = 0, cs = 0;   // cs: channel capacity, a multiple of 8
  size_t chunk_elems() const { return (size_t)(H + 2 * pad) * (W + 2 * pad) * 8; }
  size_t frame_elems() const { return chunk_elems() * (cs / 8); }
  size_t bytes() const { return frame_elems() * n * sizeof(float); }
};

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_PRELU = 2 };

// One input chunk of a split-fp16 conv whose producer left split-K partial sums instead
// of its output (ConvLaunch::fold, conv_x3 VAR 8192): the consumer's staging sums them in
// range order and applies the producer's epilogue, exactly as x3_splitk_reduce would have
// (the reduce launch is skipped).  ws == nullptr: the chunk is read from the buffer.
struct X3Fold {
  const float* ws;          // partials of this chunk: + n * fstride + m * 8 + k * sstride (range k)
  long long fstride, sstride;
  const float* bias;        // 8 values of the chunk
  const float* slope;       // 8 PReLU slopes (act == ACT_PRELU)
  float scale;              // the producer's 2^-s
  int S, act, pad_;
};

// One convolution launch.
struct ConvLaunch {
  const float* in;  int in_pad, in_cs, in_coff;
  float* out;       int out_pad, out_cs, out_coff;
  const float* wpk;            // packed weights  [co_tile][chunk][ky][kx][plane][BCO][4]
  const float* bias;           // [co_tiles*BCO]
  const float* slope;          // [co_tiles*BCO] or null
  int n, H, W;
  int ks;                      // 1, 3, 7
  int cin_chunks;              // physical input channels / 8
  int cout;                    // real output channels
  int bco;                     // output channels per block tile (32, 64, 96, 128)
  int act;
  // split-fp16 path (conv_x3.hip)
  const void* wx3 = nullptr;   // pre-split weights [co_tile][pair][ky][kx][hi|lo][h][BCO][8] fp16
  float wscale_inv = 1.f;      // 2^-s, the inverse of the per-layer weight scale
  int* range_flag = nullptr;   // raised when an output leaves the fp16 split range
  // split-K workspace (conv_x3 on grids too small to fill the GPU); null = no split
  float* ws = nullptr;
  size_t ws_floats = 0;
  int ksplit = 1;              // set by launch_conv_x3
  int allow_split = 0;         // the net's split-K switch (isl_net_set_split_k)
  unsigned long long* dbg = nullptr;   // development stamps (tools/convbench), never set by the runtime
  // Half of a following 2x2 max-pool (conv_x3 only, even W): the epilogue writes the
  // max of each horizontal pixel pair into `out` as an unpadded [n][chunk][H][W/2][8]
  // buffer (out_pad 0); launch_vpool2 then takes the max of row pairs.
  int hpool = 0;
  // The other half (conv_x3 only): `in` is such a pair-max buffer [n][chunk][2H][W][8] of
  // the pool whose H x W output this conv reads; its staging takes the max of each row
  // pair on the fly (the ring, in_pad wide, reads as zeros), so the pool kernel and its
  // output buffer are skipped.  in_pad / in_cs / in_coff describe the pooled buffer.
  int vin = 0;
  // Split-K fold (conv_x3 only).  fold: device table [cin_chunks] of X3Fold for this conv's
  // input chunks (a consumer); fold_out: this conv's across-block partial sums are consumed
  // by folding consumers, so its x3_splitk_reduce launch is skipped (a producer).
  const X3Fold* fold = nullptr;
  int fold_out = 0;

  // The fused 1x1 pair (conv_x3 VAR 16; Mconv6 -> Mconv7 of a stage, model.py:108-109):
  // cout7 > 0 makes this launch the pair.  The fields above describe Mconv6 (wx3 packed for a
  // tile of all its cout channels) with `out` / out_* describing Mconv7's output; these
  // describe Mconv7 (wx3f7 = pack_x3_f7, K in the order of Mconv6's accumulator registers).
  const void* wx3f7 = nullptr;
  const float* bias7 = nullptr;
  const float* slope7 = nullptr;
  float wscale7_inv = 1.f;
  int cout7 = 0, act7 = 0;
};

// Pixels per tile of the flattened-raster conv kernels: BPX, or fewer when the
// image is so narrow that a BPX-pixel tile's padded input row segment (which
// crosses up to (W+BPX-2)/W image rows, each adding 2*in_pad ring pixels) would
// overflow the kernel's LDS segment capacity `segcap`.
inline int tile_pixels(const ConvLaunch& c, int bpx, int segcap) {
  const int P = c.ks / 2;
  for (int t = bpx; t > 1; --t)
    if (t - 1 + 2 * c.in_pad * ((c.W + t - 2) / c.W) + 2 * P + 1 <= segcap) return t;
  return 1;
}

// Returns the block tile width (output channels) the conv kernels use for cout.
int conv_bco_for(int cout);
hipError_t launch_conv(const ConvLaunch& c, hipStream_t s);
// Winograd F(2x2,3x3) path for 3x3 layers: output channels per block tile
// (64 or 96), or 0 when cout does not fit one of them; `c.wpk` then holds
// the transformed filters [co_tile][chunk][xi 16][plane 2][BCO][4].
int wino_bco_for(int cout);
hipError_t launch_wino(const ConvLaunch& c, hipStream_t s);
// Split-fp16 (3 x fp16 MFMA = fp32-accurate) direct convolution: same tiles as
// launch_conv; x3_fits() says whether the input segment of a pixel tile fits.
// 1x1 layers with x3_wide1_layer() also carry filters packed for 256-channel tiles,
// used for a launch when x3_wide1(c with bco 256) says its grid is big enough.
bool x3_wide1_layer(int ks, int cout, int cin_phys);
bool x3_wide1(const ConvLaunch& c);
// whether launch_conv_x3 has a pooled-input (ConvLaunch::vin) variant for this launch
bool x3_vin_ok(const ConvLaunch& c);
// conv1_1 (3 input channels in one chunk, 3x3, <= 64 outputs): K packed as the 27
// real (ky, kx, c) values; c.wx3 then holds the pack_x3_rgb filters [kk][hi|lo][h][64][8].
bool x3_rgb_fits(const ConvLaunch& c);
hipError_t launch_conv_x3_rgb(const ConvLaunch& c, hipStream_t s);
double conv_x3_rgb_mfma_flops(const ConvLaunch& c);
// conv1_1 -> conv1_2 -> pair-max (conv_c12.hip): l1 = conv1_1 (rgb-packed wx3), l2 = conv1_2 with
// its hpool output
bool x3_c12_fits(const ConvLaunch& l1, const ConvLaunch& l2);
hipError_t launch_conv_x3_c12(const ConvLaunch& l1, const ConvLaunch& l2, hipStream_t s);
double conv_x3_c12_mfma_flops(const ConvLaunch& l1);
hipError_t launch_conv_x3(const ConvLaunch& c, hipStream_t s);
bool x3_fits(const ConvLaunch& c);
// whether launch_conv_x3 can run c with hpool (even W, not split across blocks)
bool x3_hpool_ok(const ConvLaunch& c);
double conv_x3_mfma_flops(const ConvLaunch& c);
// Which conv_x3 variant a launch ran (isl_net_op_info): the template's VAR bits (512 row
// union, 1024 in-block K ranges, 2048 split-K across blocks, 4096 two pairs per step,
// 32768 pooled-input staging, 65536 one input buffer), X3V_RGB for conv_x3_rgb, the tile
// (pixels / 32 at bits 20-24, output channels / 32 at bits 25-28) and the kernel radius
// (ks / 2) at bits 29-30.
constexpr int X3V_RGB = 1 << 18;
constexpr int X3V_FOLD_OUT = 1 << 19;   // a split-K producer whose reduce was folded into its consumers
constexpr int X3V_C12 = 4;              // conv1_1 -> conv1_2 -> pair-max in one launch (conv_c12.hip)
constexpr int X3V_W2 = 64;              // split-fp16 Winograd F(2x2, 3x3) (wino_f16.hip)

constexpr int x3_variant_code(int var, int ks, int bpx, int bco) {
  return (var & 0xfffff) | ((bpx / 32) << 20) | ((bco / 32) << 25) | ((ks / 2) << 29);
}
int x3_last_variant();
// whether launch_conv_x3 has a fused-pair variant for a 1x1 layer of cout6 outputs followed by
// a 1x1 layer of cout7 outputs reading all of them (VAR 16)
bool x3_fused67_fits(int cout6, int cout7);
// whether a fusable pair's launch has the grid for the fused kernel (else two launches)
bool x3_fused67_grid(const ConvLaunch& c);
// MFMA FLOPs a fused-pair launch executes (both layers, tile padding included)
double conv_x3_fused67_mfma_flops(const ConvLaunch& c);
// floats of split-K workspace launch_conv_x3 would use for c (0 = no split)
size_t x3_splitk_ws_floats(const ConvLaunch& c);
// K ranges launch_conv_x3 would use for c: S, and whether they run across blocks (split-K
// through the workspace) -- the producers a consumer can fold
int x3_split_ranges(const ConvLaunch& c, bool* across_blocks);
// whether launch_conv_x3 would run c on its generic loop (the loop that can fold)
bool x3_fold_ok(const ConvLaunch& c);
// Split-fp16 Winograd F(2x2,3x3) (wino_x3.hip): 3x3 layers with cout % 4 == 0;
// c.wx3 then holds the split transformed filters [co_tile][pair][xi][hi|lo][h][64][8].
hipError_t launch_wino_x3(const ConvLaunch& c, hipStream_t s);
double wino_x3_mfma_flops(const ConvLaunch& c);
constexpr int WINO_X3_BCO = 64;
// Split-fp16 Winograd F(2x2, 3x3) on 64-channel x 64-tile blocks (wino_f16.hip): 3x3 layers with
// cout % 64 == 0, no fused pool / pooled input / fold, >= 32 tiles per row, > 1024 pixels per
// frame; c.wx3 holds the pack_wino_f16 filters and c.wscale_inv their 2^-s.
bool wino_f16_fits(const ConvLaunch& c);
hipError_t launch_wino_f16(const ConvLaunch& c, hipStream_t s);
double wino_f16_mfma_flops(const ConvLaunch& c);
// FLOPs the matrix cores execute for one launch (tile padding included)
double conv_mfma_flops(const ConvLaunch& c);
double wino_mfma_flops(const ConvLaunch& c);

hipError_t launch_maxpool2(const Act& in, const Act& out, int C, hipStream_t s);
// adds 1 to *trips when *flag is set (stream-ordered range-guard count)
hipError_t launch_range_count(const int* flag, unsigned long long* trips, hipStream_t s);
// second half of a fused 2x2 max-pool: row pairs of a horizontally pooled buffer
// (ConvLaunch::hpool, [n][chunk][H][W/2][8]) into the padded next buffer
hipError_t launch_vpool2(const Act& half, const Act& out, int C, hipStream_t s);
hipError_t launch_pack_nchw(const float* x, int n, int C, int h, int w, const Act& out, hipStream_t s);
hipError_t launch_unpack_nchw(const Act& in, int coff, int C, float* y, hipStream_t s);
// Pre-processing of a batch of images described by a device table of entries
// (preprocess_entry: byte offset of the image in `frames`, its size, the
// resized size and 1/fx); row_bytes = bytes per row of the frame array.
hipError_t launch_preprocess_tab(const uint8_t* frames, long long row_bytes, const void* d_tab, int n,
                                 const Act& out, hipStream_t s);
size_t preprocess_entry_bytes();
void preprocess_entry(void* dst, long long off, int sh, int sw, int rh, int rw, double scale);

struct MapSrc {            // one single-stage cubic resize, sampled per output element
  const float* base;       // element (f, c, y, x) at base + f*fs + chan(c) + y*ys + x*xs,
  long long fs, cstr, ys, xs;   //   chan(c) = (c >> cshift) * cbig + (c & (2^cshift - 1)) * cstr
  long long cbig;          // chunk stride of a chunked (arena) map; planar maps: cshift = 30, cbig = 0
  int cshift;
  int sh, sw;              // source size (tap clamping)
  int dh, dw;              // destination size of this resize
  double scy, scx;         // source pixels per destination pixel (1/inv_scale)
  int cn;                  // channels of the image OpenCV resized (SIMD body / tail split)
  int identity;            // dsize == ssize: plain copy
};

void set_error(const std::string& msg);


}  // namespace isl

struct isl_net;
namespace isl {
int net_kind(const isl_net* net);
int net_device(const isl_net* net);
// low-resolution output `which` (0 = out0 / PAF, 1 = out1 / heat) of the last run, as a MapSrc
int net_low_res(isl_net* net, int which, MapSrc* m);
// grow-only device scratch owned by the net (nullptr + error on failure)
void* net_scratch(isl_net* net, size_t bytes);
size_t net_scratch_size(const isl_net* net);
// streams on which isl_hand_post_crops runs its crops side by side, forked from and
// joined back into the caller's stream; a grow-only scratch per lane
constexpr int ISL_POST_LANES = 4;
struct PostLanes {
  hipStream_t stream[ISL_POST_LANES];
  hipEvent_t fork, join[ISL_POST_LANES];
  void* scratch[ISL_POST_LANES];
  size_t bytes[ISL_POST_LANES];
  // the batch's stage-1 maps (written on the caller's stream, read by the lanes): a buffer
  // of their own, released by `mid_free` (recorded on the caller's stream after the lanes
  // joined); the next writer waits on it, whatever stream it runs on
  void* mid;
  size_t mid_bytes;
  hipEvent_t mid_free;
  bool mid_used;
};
// created on first use (nullptr + error on failure), destroyed with the net
PostLanes* net_post_lanes(isl_net* net);
}  // namespace isl
