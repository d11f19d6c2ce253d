// Per-GPU streaming session: frame source -> colour conversion (+ scale) -> H.264 encode,
// driven on HIP streams (SURVEY.md C41 frame pool, C44 pipeline scheduler).
//
// Replaces the reference's GStreamer pipeline `ximagesrc ! cudaupload ! cudaconvert !
// nvh264enc` (selkies, launched from selkies-gstreamer-entrypoint.sh:44-47): the desktop
// framebuffer lives in HBM (synthetic source) or is uploaded from pinned host memory
// (X11 SHM capture), and only the encoded bitstream crosses PCIe.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <deque>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "../codec/h264_encoder.h"
#include "../codec/video_encoder.h"
#include <string>
#include "../kernels/pixel.h"

namespace mx {

// HBM ring of BGRx frames with generation counters (use-after-recycle detection).
class FramePool {
   public:
    FramePool(int width, int height, int slots);
    ~FramePool();
    FramePool(const FramePool&) = delete;
    FramePool& operator=(const FramePool&) = delete;
    int width() const { return w_; }
    int height() const { return h_; }
    int pitch() const { return pitch_; }
    int slots() const { return (int)buf_.size(); }
    // Acquire the next slot for writing; returns its index and bumps its generation.
    int acquire();
    uint8_t* data(int slot) const { return buf_[slot]; }
    uint64_t generation(int slot) const { return gen_[slot]; }
    // True if `slot` still holds generation `gen` (not recycled).
    bool valid(int slot, uint64_t gen) const { return gen_[slot] == gen; }

   private:
    int w_, h_, pitch_;
    std::vector<uint8_t*> buf_;
    std::vector<uint64_t> gen_;
    int next_ = 0;
    uint64_t counter_ = 0;
};

struct SessionConfig {
    int width = 1920;       // desktop (capture) size
    int height = 1080;
    int out_width = 0;      // encode size; 0 = same as desktop (no scaling)
    int out_height = 0;
    int fps = 60;
    int noise = 1;          // synthetic animated-noise panel
    int content = 0;        // synthetic source: 0 desktop, 1 motion content (pan + video panel, pix::SynthParams),
                            // 2 sub-sample motion (2.5 / 0.75 px per frame pan, zooming video panel)
    int pool_slots = 5;     // > encoder pipeline depth (<= kMaxDepth)
    int use_graph = 0;      // replay the per-frame chain as a hipGraph (measured slower than eager
                            // launches on ROCm 7.2 for this chain: profiles/r01_graph)
    int fake_clock = 0;     // barcode timestamp = frame_id * 1e6 / fps (deterministic streams for tests)
    std::string codec = "h264";  // "h264" (mxh264enc) or "hevc" / "h265" (mxh265enc)
    // optional quality report: luma PSNR with a rectangle (encoded-picture coordinates) left
    // out, e.g. the incompressible noise panel of the synthetic desktop; mask_x1 <= mask_x0 = off
    int mask_x0 = 0, mask_y0 = 0, mask_x1 = 0, mask_y1 = 0;
    int scale_valu = 0;     // 1: the LDS/VALU Lanczos kernel instead of the matrix-core one
    // pipeline depth > 1: render + convert each frame on a capture stream into its own NV12
    // buffer, so frame n+1's capture overlaps frame n's analysis.  -1 = H.264 and HEVC (1080p H.264:
    // 9,040 -> 10,125 fps, profiles/r04_capture; 4K HEVC: 2,176 -> 2,277 fps once its entropy
    // streams leave the capture stream a hardware queue of its own -- sharing the analysis queue it
    // had cost 2,272 -> 1,633 in round 4, profiles/r06_streams), 1 = every codec (VP8 too), 0 = one
    // analysis stream
    int capture_stream = -1;
    h264::EncoderConfig enc;  // width/height overwritten from out size
};

struct FrameResult {
    uint32_t frame_id = 0;
    int64_t t_capture_us = 0;  // CLOCK_MONOTONIC us when the frame was rendered/captured
    int64_t t_encoded_us = 0;  // CLOCK_MONOTONIC us when the access unit was available
    double gpu_ms = 0;         // device time render->bitstream (events)
    int idr = 0;
    int qp = 0;
    double psnr_y = 0, psnr_u = 0, psnr_v = 0;  // encoder reconstruction vs source (dB, cap 99)
    double psnr_y_masked = 0;                   // luma PSNR outside SessionConfig::mask_* (0 = off)
    int deblocked = 0;                          // H.264: the in-loop filter ran on this picture
    int db_coherent = 0, db_moving = 0;         // H.264: the picture's adaptive-filter classes (h264_deblock.h)
    std::vector<uint8_t> au;
};

class Session;
// Paced serving load: K sessions at `fps` for `seconds`, driven by `threads` host threads (session
// i on thread i % threads, one frame in flight per session).  Every 1/fps slot each thread
// submits a frame on each of its sessions, then collects them; a slot is late when any thread
// finished it after the next slot's start.  Latency = capture -> access unit on the host.
// idr_slot >= 0: in that slot every session codes a forced IDR picture (an IDR storm: viewers
// joining together, a PLI burst after a network event).
struct PacedStats {
    int slots = 0;
    int late_slots = 0;
    std::vector<double> lat_ms;  // every frame of every session (slot order)
    int idr_late = 0;            // the storm slot overran
    std::vector<double> idr_lat_ms;  // the storm slot's frames
};
PacedStats run_sessions_paced(const std::vector<Session*>& sessions, int fps, double seconds, int threads,
                              int idr_slot = -1);
// Drives several sessions concurrently, one host thread per session (submit / collect with up
// to `depth` frames in flight each): the per-frame launch sequence is host work, so one
// thread interleaving K sessions leaves the GPU waiting on it.  Returns each session's
// results in frame order.  The calling thread's HIP device is used by every worker.
std::vector<std::vector<FrameResult>> run_sessions(const std::vector<Session*>& sessions, int n_frames, int depth);

class Session {
   public:
    explicit Session(const SessionConfig& cfg);
    ~Session();
    Session(const Session&) = delete;
    Session& operator=(const Session&) = delete;

    // Synthetic desktop frame -> encode.  `submit` enqueues, `collect` waits.
    void submit_synthetic(bool force_idr = false);
    int in_flight() const { return (int)inflight_.size(); }
    int depth() const { return depth_; }
    // Externally captured BGRx frame (host memory, e.g. X11 SHM) -> upload -> encode.
    void submit_bgrx(const uint8_t* host_bgrx, int host_pitch, bool force_idr = false);
    // Page-locks a host buffer the capture writes frames into (e.g. the XShm segment):
    // submit_bgrx from inside it is a direct 2D DMA, with no copy into the staging buffer, and
    // returns once the DMA has read the frame (the buffer may then be overwritten).
    void register_host_buffer(const void* p, size_t bytes);
    // submit_bgrx from a raw host address whose readable extent is `bytes`: throws
    // std::invalid_argument unless the frame span (pitch * (height - 1) + width * 4) fits.
    void submit_bgrx_span(const uint8_t* host_bgrx, int host_pitch, size_t bytes, bool force_idr = false);
    // Damage-driven capture (XDamage): only the row bands [y0, y1) that changed since the last
    // submit are DMA'd from the host frame into a device-resident copy of the screen, which is
    // then copied into the frame-pool slot on the device.  The first call (and any call after
    // invalidate_screen()) uploads the whole frame.  An empty band list re-encodes the resident
    // screen without reading host memory.  A static desktop costs no PCIe traffic (at 1080p60 a
    // full-frame upload is 0.5 GB/s per session, so 200 sessions would exceed a x16 link).
    void submit_bgrx_damage(const uint8_t* host_bgrx, int host_pitch, size_t bytes,
                            const std::vector<std::pair<int, int>>& bands, bool force_idr = false);
    void invalidate_screen() { screen_valid_ = false; }
    // host bytes DMA'd by submit_bgrx_damage so far (bands + first full frames)
    uint64_t damage_bytes_uploaded() const { return damage_bytes_; }
    FrameResult collect();
    FrameResult step(bool force_idr = false) {
        submit_synthetic(force_idr);
        return collect();
    }

    void set_cursor(int x, int y) {
        cursor_x_ = x;
        cursor_y_ = y;
    }
    void request_idr() { enc_->rc().request_idr(); }
    void set_bitrate(int kbps) { enc_->rc().set_bitrate(kbps); }
    const SessionConfig& config() const { return cfg_; }
    hipStream_t stream() const { return stream_; }
    VideoEncoder& encoder() { return *enc_; }
    FramePool& pool() { return *pool_; }
    // Device pointers of the NV12 frame fed to the encoder (tests / wall composite).
    // (the most recently submitted frame's: one buffer per frame in flight)
    const uint8_t* nv12_y() const { return nv12_y_[last_k_]; }
    const uint8_t* nv12_uv() const { return nv12_uv_[last_k_]; }
    int nv12_pitch() const { return enc_->pitch(); }
    static int64_t now_us();

    int graphs_built() const { return graphs_built_; }
    bool capture_stream_active() const { return cap_stream_ != nullptr; }

   private:
    void convert(int slot, hipStream_t st, uint64_t* ts = nullptr);
    // stamp: the conversion stores the frame's start clock (capture paths; the synthetic path's
    // render stamps it)
    void convert_and_encode(int slot, bool force_idr, bool stamp);
    void encode_converted(bool force_idr);  // encoder submit + masked SSE of NV12 buffer cur_k_
    pix::SynthParams synth_params();
    hipGraphExec_t capture_on(hipStream_t st, const std::function<void()>& body);
    void capture_frame_graphs(int slot, bool idr, hipGraphExec_t* ga, hipGraphExec_t* ge);

    SessionConfig cfg_;
    hipStream_t stream_ = nullptr;
    std::unique_ptr<FramePool> pool_;
    std::unique_ptr<VideoEncoder> enc_;
    static constexpr int kMaxDepth = 4;  // frames in flight per session (encoder pipeline depth)
    // NV12 encoder input per frame in flight: the buffer of frame n is rewritten by frame
    // n + depth, whose submit follows collect(n) (analysis, entropy and masked SSE complete)
    uint8_t* nv12_y_[kMaxDepth] = {};
    uint8_t* nv12_uv_[kMaxDepth] = {};
    int cur_k_ = 0, last_k_ = 0;  // frame being submitted / last submitted (begin_frame)
    hipStream_t cap_stream_ = nullptr;    // SessionConfig::capture_stream with depth > 1
    hipEvent_t ev_conv_[kMaxDepth] = {};  // conversion done -> analysis stream
    uint8_t* staging_[kMaxDepth] = {};  // pinned upload buffers (one per frame in flight)
    // Lanczos tables (device) when out size != desktop size
    bool scale_ = false;
    pix::LanczosTables lt_{};
    void* lt_mem_ = nullptr;
    void* lt_mf_mem_ = nullptr;  // MFMA scaler fragment tables
    std::vector<std::pair<const uint8_t*, size_t>> host_regs_;  // register_host_buffer ranges
    hipEvent_t ev_upload_ = nullptr;
    hipStream_t upload_stream_ = nullptr;  // zero-copy DMA from registered capture buffers
    uint8_t* screen_ = nullptr;  // device-resident screen (submit_bgrx_damage), pool pitch
    bool screen_valid_ = false;
    uint64_t damage_bytes_ = 0;
    void ensure_upload_stream();
    void encode_uploaded(int slot, int k, bool force_idr);  // tail of the upload-stream paths
    // frames in flight (pipeline depth 1..kMaxDepth): per-frame start event / staging buffer
    struct Inflight {
        uint32_t frame_id;
        int64_t t_capture;
        int k;     // index into ev_start_ / staging_
        int slot;  // frame-pool slot (index into ts_)
    };
    std::deque<Inflight> inflight_;
    hipEvent_t ev_start_[kMaxDepth] = {};  // encoders without device clock stamps only
    // device clock at each frame's first kernel (render or conversion), per pool slot (mapped pinned):
    // with an encoder's end stamp it gives the frame's GPU time without events between kernels
    uint64_t* ts_ = nullptr;
    bool devclk_ = false;
    double clock_khz_ = 100000;
    // masked-PSNR accumulators (device) + their host copies, one per frame in flight
    unsigned long long* mask_dev_ = nullptr;
    unsigned long long* mask_host_ = nullptr;  // mapped pinned, one word per frame in flight
    unsigned int* mask_counter_ = nullptr;     // single-pass reduction counters (device)
    int mask_stride_ = 0;
    hipEvent_t ev_mask_[kMaxDepth] = {};
    bool masked() const { return cfg_.mask_x1 > cfg_.mask_x0 && cfg_.mask_y1 > cfg_.mask_y0; }
    bool mask_in_encoder_ = false;  // H.264: the encoder reports the masked distortion itself
    void enqueue_mask_sse(int k);
    void mask_rect_mb(int r[4]) const;  // mask rectangle aligned out to macroblocks, clipped
    int next_k_ = 0;
    int depth_ = 1;
    // hipGraph replay: pinned + device synth parameters, one executable graph per
    // (pool slot, frame type) -- the only things that change the captured node arguments
    pix::SynthParams* synth_host_ = nullptr;
    pix::SynthParams* synth_dev_ = nullptr;
    uint8_t* synth_bg_ = nullptr;  // static layer of the synthetic desktop (rendered once)
    std::vector<hipGraphExec_t> graphs_;
    int graphs_built_ = 0;
    uint32_t frame_id_ = 0;  // id of the next submitted frame
    int64_t t0_us_ = 0;
    // host-side time per frame (MXDESK_HOST_TIMING=1 prints the means when the session ends):
    // submit, collect (wait for the GPU), collect (after the wait)
    double ht_submit_ = 0, ht_wait_ = 0, ht_post_ = 0;
    int64_t ht_n_ = 0;
    int64_t t_capture_ = 0;
    int cursor_x_ = -1, cursor_y_ = -1;
    int begin_frame(int slot);  // reserve an in-flight entry for a frame in pool slot `slot`, returns its k
};

// Host-side Lanczos-3 table generation (shared with the Python reference in tests).
void make_lanczos_table(int in_size, int out_size, std::vector<int>& start, std::vector<float>& weights, int& taps);

}  // namespace mx
