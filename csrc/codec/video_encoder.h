// Codec-independent interface of the GPU encoders the streaming Session drives
// (GpuH264Encoder, GpuHevcEncoder).  Selected by SessionConfig::codec, the equivalent of
// the reference's WEBRTC_ENCODER element choice (reference Dockerfile:210).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "h264_gpu.h"

namespace mx {
namespace h264 {
class EncoderCommon;
struct FrameStats;
}  // namespace h264

class VideoEncoder {
   public:
    virtual ~VideoEncoder() = default;
    virtual const char* codec() const = 0;  // "h264" / "hevc"
    virtual const h264::Geometry& geometry() const = 0;
    virtual int pitch() const = 0;
    virtual int depth() const = 0;
    virtual void submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr) = 0;
    virtual const std::vector<uint8_t>& collect() = 0;
    virtual const h264::FrameStats& last_stats() const = 0;
    virtual h264::EncoderCommon& rc() = 0;  // rate control / IDR requests
    virtual const uint8_t* recon_y() const = 0;
    virtual const uint8_t* recon_uv() const = 0;
    virtual hipEvent_t done_event() const = 0;
    // device_clock(): the encoder stamps its frames with the device wall clock (no timing events);
    // last_t_end() is the end stamp of the last collected frame (device_clock_khz() ticks per ms)
    virtual bool device_clock() const { return false; }
    virtual uint64_t last_t_end() const { return 0; }
    // completion event of the oldest frame in flight (the next collect() waits for it)
    virtual hipEvent_t pending_done_event() const = 0;
    // split form for hipGraph capture (pipeline depth 1: enqueue_body on one stream)
    virtual bool prepare(bool force_idr) = 0;
    virtual void enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) = 0;
    virtual void record_start() = 0;
    virtual void record_done() = 0;
    // depth-2 graph form: the frame state upload + analysis kernels on the session stream and the
    // entropy kernels on entropy_stream(), captured as two graphs per (frame slot, encoder slot,
    // picture type) and linked per frame by link_entropy() (analysis event -> entropy stream).
    // supports_split() false: eager submission only.
    virtual bool supports_split() const { return false; }
    // FrameStats::sse_masked / masked_pixels are filled by the encoder itself (no separate pass)
    virtual bool masked_sse_in_encoder() const { return false; }
    virtual int prep_slot() const { return 0; }
    virtual hipStream_t entropy_stream() const { return nullptr; }
    virtual void enqueue_analysis(bool idr, const uint8_t* src_y, const uint8_t* src_uv) { (void)idr; (void)src_y; (void)src_uv; }
    virtual void enqueue_entropy() {}
    virtual void link_entropy() {}
    // false: the reference half-pel planes are interpolated on the analysis stream itself (the
    // session converts the next frame on a capture stream, so nothing on the analysis stream
    // would overlap a side-stream interpolation -- it would only add two cross-queue hand-offs)
    virtual void set_hpel_side_stream(bool on) { (void)on; }
    // every launch this encoder queued on a helper thread has been issued (before the caller
    // captures or replays graphs on the encoder's streams)
    virtual void quiesce() {}
    // The next submit's source is ready when `ev` completes: the encoder waits for it on its
    // analysis stream right before the first kernel that reads the source.  Returns false if
    // the encoder does not take the event (the caller then waits before submitting).
    virtual bool set_input_event(hipEvent_t ev) { (void)ev; return false; }
};

}  // namespace mx
