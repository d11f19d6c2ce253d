// Pixel kernels (SURVEY.md C40 synthetic desktop, C42 CSC/scale, K7 composite).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>
#include <stdint.h>

namespace mx {
namespace pix {

// Parameters of the synthetic desktop frame (animated noise + gears + scrolling text +
// moving window + frame-id/timestamp barcode).
struct SynthParams {
    int width, height;      // frame size
    int pitch;              // bytes per BGRx row
    uint32_t frame_id;      // encoded in the barcode
    uint32_t timestamp_us;  // encoded in the barcode (capture clock, low 32 bits)
    float t;                // animation time in seconds
    int origin_x, origin_y; // offset of this frame inside a larger wall (tile rendering)
    int wall_w, wall_h;     // full desktop size (== width/height for a single session)
    int noise;              // 1 = animated-noise panel on
    int cursor_x, cursor_y; // remote cursor position (-1 = hidden)
    uint64_t* ts = nullptr; // if set: device wall clock at the render's start (frame GPU time)
    // 0: the desktop (static windows + animated elements); 1: motion content -- the whole desktop
    // pans (3 px right, 1 px down per frame at 60 fps, wrapping) under a screen-fixed video-like
    // panel of smooth, colourful, non-rigidly moving texture (kVideo* rectangle), as games and
    // video playback look to the encoder; the barcode stays put.  2: sub-sample motion -- the pan
    // moves 2.5 px right and 0.75 px down per frame (bilinear resampling of the desktop) and the
    // video panel's texture zooms (a scaled video), so the motion is fractional
    int content = 0;
};
// video panel of the motion content, fractions of the wall (screen coordinates)
constexpr float kVideoX = 0.60f, kVideoY = 0.56f, kVideoW = 0.34f, kVideoH = 0.36f;

// Barcode geometry: 64 bits (frame_id, timestamp_us), 8x8-pixel cells, two rows of 32
// cells, drawn at the top-left of the desktop with a one-cell quiet zone.
constexpr int kBarCell = 8;
constexpr int kBarX = 8, kBarY = 8;

// static_bg: the static-layer cache rendered by launch_synth_static for the same size /
// pitch / origin (pixels outside the animated elements are copied from it), or nullptr.
void launch_synth(uint8_t* bgrx, const SynthParams& p, hipStream_t stream, const uint8_t* static_bg = nullptr);
void launch_synth_static(uint8_t* bgrx, const SynthParams& p, hipStream_t stream);
// Same, reading the parameters from device memory (hipGraph replay; width/height fix the grid).
void launch_synth_dev(uint8_t* bgrx, const SynthParams* d_params, int width, int height, hipStream_t stream,
                      const uint8_t* static_bg = nullptr);

// BGRx -> NV12 (BT.709 limited range), padding the output to (coded_w, coded_h) by edge
// replication.  Output Y plane pitch = UV plane pitch = out_pitch.
// ts: if set, the device wall clock at the kernel's start is stored there (frame GPU time).
void launch_bgrx_to_nv12(const uint8_t* bgrx, int in_pitch, int w, int h, uint8_t* y, uint8_t* uv, int out_pitch,
                         int coded_w, int coded_h, hipStream_t stream, uint64_t* ts = nullptr);

// Fused separable Lanczos-3 resample (in_w x in_h -> out_w x out_h) + BT.709 CSC into
// NV12, LDS-tiled.  `weights` from make_lanczos_tables (device memory).
// MFMA form of the scaler (see build_scale_frags): per 32-column group the first staged
// input column and K-step count, per 32-row group the first input row, row-block count and
// row span, and the weights pre-laid-out as f16 MFMA operand fragments.
struct ScaleMfma {
    const int* gx = nullptr;    // [ngx][2] kabs, nks
    const int* gy = nullptr;    // [ngy][3] ylo, nrb, nr
    const void* fh = nullptr;   // [ngx][kMaxKs][64 lanes] 8 x f16 horizontal weight fragments
    const void* fv = nullptr;   // [ngy][kMaxRb][2][64 lanes] 8 x f16 vertical weight fragments
    int lds_cols = 0, lds_rows = 0, ngx = 0, ngy = 0;
    int nk = 0;       // K-steps k_scale_mfma is instantiated for (max over the groups, rounded up)
    int nrb_max = 0;  // most 32-row input blocks of a row group
    // strip form (k_scale_strip: `strip` consecutive 32-row tiles per workgroup, 0 = unavailable):
    // per tile (first input row of its strip, first block | blocks << 8 relative to it, 0) and the
    // vertical fragments against those strip-relative 32-row blocks
    const int* gy2 = nullptr;   // [ngy][3]
    const void* fv2 = nullptr;  // [ngy][kMaxRb][2][64 lanes]
    int strip = 0;
    bool force_strip = false;  // use the strip form (else only with MXDESK_SCALER=strip)
};
struct LanczosTables {
    int out_w, out_h, taps_x, taps_y;
    const int* x0;      // [out_w] first input column
    const float* wx;    // [out_w * taps_x]
    const int* y0;      // [out_h]
    const float* wy;    // [out_h * taps_y]
    ScaleMfma mf{};     // gx == nullptr: LDS/VALU kernel
};

// Host side of the MFMA scaler: fragment tables for one (in, out, coded) geometry, packed in
// one blob (`blob`) that upload_scale_frags copies to the device.  Returns false when the
// scale factor is outside what the MFMA kernel's register tiles hold (then the VALU kernel runs).
struct ScaleFragsHost {
    std::vector<uint8_t> blob;
    size_t off_gx = 0, off_gy = 0, off_fh = 0, off_fv = 0, off_gy2 = 0, off_fv2 = 0;
    int lds_cols = 0, lds_rows = 0, ngx = 0, ngy = 0, strip = 0, nk = 0, nrb_max = 0;
};
bool build_scale_frags(int in_w, int in_h, int out_w, int out_h, int coded_w, int coded_h,
                       const std::vector<int>& x0, const std::vector<float>& wx, int tx, const std::vector<int>& y0,
                       const std::vector<float>& wy, int ty, ScaleFragsHost& out);
// Copies the blob to `dev` (hipMalloc'ed here; caller frees) and fills `mf`.
void upload_scale_frags(const ScaleFragsHost& h, void** dev, ScaleMfma& mf);
void launch_scale_to_nv12(const uint8_t* bgrx, int in_pitch, int in_w, int in_h, const LanczosTables& t, uint8_t* y,
                          uint8_t* uv, int out_pitch, int coded_w, int coded_h, hipStream_t stream,
                          uint64_t* ts = nullptr);

// Luma squared error between two planes over [0,w) x [0,h) excluding the rectangle
// [mx0,mx1) x [my0,my1) (quality report with a panel masked out), in one dispatch: `part`
// holds sse_masked_blocks(w, h) partials, `counter` is a zero-initialised device uint that the
// kernel leaves at zero, and the total is stored to `host_out` (mapped pinned memory).
int sse_masked_blocks(int w, int h);
void launch_sse_masked(const uint8_t* a, const uint8_t* b, int pitch, int w, int h, int mx0, int my0, int mx1,
                       int my1, unsigned long long* part, unsigned int* counter, unsigned long long* host_out,
                       hipStream_t stream);

// Place cols x rows packed NV12 tiles (rank order, each tw x th: Y rows then UV rows, pitch tw)
// into the wall's NV12 planes (pitch `pitch`) in one launch (tiled-wall composite, K7).
void launch_composite_nv12(const uint8_t* tiles, int tw, int th, int cols, int rows, uint8_t* y, uint8_t* uv,
                           int pitch, hipStream_t stream);

// Copy a BGRx tile into a larger BGRx frame at (dx, dy) (tiled-wall composite).
void launch_composite(const uint8_t* tile, int tile_pitch, int tw, int th, uint8_t* dst, int dst_pitch, int dx, int dy,
                      hipStream_t stream);

}  // namespace pix
}  // namespace mx
