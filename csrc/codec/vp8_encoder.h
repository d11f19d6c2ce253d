// VP8 encoders (RFC 6386): GpuVp8Encoder (HIP analysis -- motion search shared with H.264,
// transforms, quantisation, reconstruction -- plus boolean-coded partitions written by host
// threads, one per token partition) and CpuVp8Encoder (the same decisions serially; the bit-exact
// oracle for the GPU path and the no-GPU fallback).  Selected by WEBRTC_ENCODER=vp8enc, the
// reference's libvpx choice (reference README.md:21,35).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <array>
#include <condition_variable>
#include <deque>
#include <exception>
#include <memory>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "h264_deblock.h"
#include "h264_encoder.h"
#include "h264_mb.h"
#include "video_encoder.h"
#include "vp8_core.h"

namespace mx {
namespace vp8 {

// RFC 6386 section 7 boolean entropy encoder (libvpx's carry-propagating form).
class BoolEncoder {
   public:
    explicit BoolEncoder(std::vector<uint8_t>& out) : out_(out) {}
    // The RFC's one-bit-at-a-time normalisation, batched: the shift count comes from the leading
    // zeros of the range and the whole shift is applied at once to a 64-bit low end that keeps
    // up to 38 pending bits; whole bytes leave once 32 bits are pending (where the per-bit form
    // emits its byte, so the byte alignment is the same), each after the carry that reached
    // above them (one bit: low + range never exceeds the interval) went into the bytes already
    // written.  The coded bit selects with masks instead of a branch (the bits of a picture are
    // close to random: a branch on them mispredicts).  Same bits as the per-bit form (tests:
    // libwebp key frames, the in-tree decoder, GPU == CPU streams).
    void put(int prob, int bit) {
        const uint32_t split = 1 + (((range_ - 1) * (uint32_t)prob) >> 8);
        const uint32_t m = 0u - (uint32_t)(bit != 0);
        low_ += split & m;
        range_ = ((range_ - split) & m) | (split & ~m);
        const int s = __builtin_clz(range_) - 24;  // range_ in [1, 255]: shifts to bring it to [128, 255]
        range_ <<= s;
        low_ <<= s;
        pend_ += s;
        if (pend_ >= 32) emit();
    }
    void literal(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; --i) put(128, (v >> i) & 1);
    }
    void flush() {
        for (int i = 0; i < 32; ++i) put(128, 0);
    }

   private:
    void emit() {  // pend_ >= 32: the bytes above the low 24 pending bits go out
        while (pend_ >= 32) {
            if (low_ >> pend_) {  // carry into the bytes already written
                for (size_t i = out_.size(); i-- > 0;) {
                    if (out_[i] == 255) {
                        out_[i] = 0;
                    } else {
                        ++out_[i];
                        break;
                    }
                }
                low_ &= (uint64_t(1) << pend_) - 1;
            }
            pend_ -= 8;
            out_.push_back((uint8_t)(low_ >> pend_));
            low_ &= (uint64_t(1) << pend_) - 1;
        }
    }
    std::vector<uint8_t>& out_;
    uint32_t range_ = 255;
    uint64_t low_ = 0;  // pend_ pending bits (bit pend_: a carry not yet added to out_)
    int pend_ = 8;      // the 8-bit window counts: the first byte leaves after 24 shifts
};

struct FrameDesc {
    bool key;
    int width, height, mb_w, mb_h;
    int qindex;
    int log2_parts;  // token partitions: 1 << log2_parts
    bool segmented = false;          // inter frames with aq >= 3: segment map + segment quantisers
    int seg_qindex[kNumSegs] = {0, 0, 0, 0};
    int lf_level[kNumSegs] = {0, 0, 0, 0};  // loop-filter level per segment ([0]: unsegmented); 0 = off
};
// Segment quantiser indices of an inter frame at frame QP `qp` (the classes' QPs of aq3_mb_qp).
inline void segment_qindices(int qp, int aq, int out[kNumSegs]) {
    for (int s = 0; s < kNumSegs; ++s) out[s] = qindex_for_qp(h264::aq3_mb_qp(qp, tclass_of_seg(s), aq));
}

// Per-segment loop-filter levels of a frame (all zero: the filter is off): from each segment's
// quantiser (lf_level_for), the static segment (identical source, zero vector) unfiltered.
inline void lf_levels(bool on, bool segmented, int qindex, const int seg_qindex[kNumSegs], int num, int out[kNumSegs]) {
    for (int s = 0; s < kNumSegs; ++s)
        out[s] = !on ? 0 : (!segmented ? lf_level_for(qindex, num) : (s == kSegStatic ? 0 : lf_level_for(seg_qindex[s], num)));
}
// lf_level_for's numerator: MXDESK_VP8_LF_NUM (tuning), else kLfNumDefault
int lf_num_from_env();

// Token branch statistics of the last coded frame of one type (13.4): the coefficient probability
// updates of the next frame of that type are planned from them, so coding needs no separate
// counting pass over the tokens.
// Frames whose bitstreams may be written at once (GPU encoder pipeline depth); also the distance
// from the frame whose branch statistics plan a frame's probability updates.
constexpr int kStatsLag = 4;

struct TokenStats {
    std::vector<std::array<uint32_t, 2>> n;  // [1056] (zeros, ones) per probability
    bool valid = false;
    // diagnostics of the last write_frame: first partition / sum over token partitions (host us)
    double us_first = 0, us_tokens = 0;
};

// Writes a complete VP8 frame (frame tag, key-frame header, first partition, token partitions)
// from per-macroblock records and levels.  `levels(i)` returns macroblock i's 400 levels (only
// read for macroblocks with nz != 0).  Token partitions are coded concurrently on `run_parallel`.
// stats (may be null: no probability updates, e.g. rate-control probes): in, the previous frame's
// branch statistics of this frame type; out, this frame's.
void write_frame(const FrameDesc& f, const Vp8Mb* mbs, const std::function<const int16_t*(int)>& levels,
                 std::vector<uint8_t>& out,
                 const std::function<void(int, const std::function<void(int)>&)>& run_parallel,
                 TokenStats* stats = nullptr);

// Near / nearest / best motion vectors of macroblock (mbx, mby) (RFC 6386 find_near_mvs, with
// the decoder's clamping); every macroblock of the picture is inter (P frames).  cnt[4] out.
void find_near_mvs(const Vp8Mb* mbs, int mb_w, int mb_h, int mbx, int mby, int near_mv[3][2], int cnt[4]);
// Legal full-sample vector range of a macroblock: the decoder never clamps vectors inside it.
MXV8 void mv_bounds(int mb_w, int mb_h, int mbx, int mby, int* lo_x, int* hi_x, int* lo_y, int* hi_y) {
    *lo_x = -(mbx * 16 + 16) + 3;
    *hi_x = (mb_w - 1 - mbx) * 16 + 16 - 3;
    *lo_y = -(mby * 16 + 16) + 3;
    *hi_y = (mb_h - 1 - mby) * 16 + 16 - 3;
}

// The inter vector of a macroblock in 1/8 samples from the motion search's quarter-sample vector
// (luma vectors are quarter-sample in VP8: even 1/8 phases), clamped to mv_bounds.
MXV8 void inter_vector(int qx, int qy, int lo_x, int hi_x, int lo_y, int hi_y, int* mvx, int* mvy) {
    const int vx = 2 * qx, vy = 2 * qy;
    *mvx = vx < 8 * lo_x ? 8 * lo_x : (vx > 8 * hi_x ? 8 * hi_x : vx);
    *mvy = vy < 8 * lo_y ? 8 * lo_y : (vy > 8 * hi_y ? 8 * hi_y : vy);
}

// Rate-distortion residual drop of noise-like inter macroblocks (the rule of the H.264 encoder's
// aq 2, h264_mb.h drop_residual): a macroblock whose prediction residual stays above 32 per luma
// sample on average keeps its residual only if coding it lowers the luma SSE by more than
// lambda * (estimated bits); else it goes out as prediction only (no tokens, skipped).
// Incompressible content (the bench desktop's noise panel, video) otherwise takes the bits the
// rest of the picture needs: VP8 has no per-macroblock quantiser here to send it coarser.
// bits: sum over the 16 luma blocks (AC levels) and Y2 of 2 + 6 * non-zero levels.
MXV8 bool vp8_drop_residual(uint32_t lsad, long long d_pred, long long d_coded, uint32_t bits, int lambda) {
    return lsad > 256u * 32 && d_pred - d_coded < (long long)lambda * (long long)bits;
}
MXV8 uint32_t vp8_block_bits(int nz) { return nz ? 2u + 6u * (uint32_t)nz : 0u; }

// Loop-filter decision per frame (EncoderConfig::deblock: 0 off, 1 on, 2 or -1 (the VP8 default)
// adaptive).  Adaptive is the H.264 encoder's rule (h264_deblock.h db_auto_decide: filter when the
// moving macroblocks move coherently -- pans, scrolls, video -- not for a still desktop, whose text
// the filter only blurs) on the vectors of the inter frame kStatsLag frames back: the newest frame
// whose records the host holds when a frame is prepared at any pipeline depth, so the CPU and GPU
// encoders decide alike.  A key frame keeps the last decision.
class LfDecision {
   public:
    explicit LfDecision(int mode) : mode_(mode) {}
    // the decision for frame `fidx`, before it is analysed (called in frame order)
    bool decide(long long fidx, bool key) {
        if (mode_ != 2) return on_ = mode_ == 1;
        const Rec& r = ring_[fidx % kStatsLag];
        if (!key && r.valid && r.fidx == fidx - kStatsLag) on_ = h264::db_auto_decide(r.c, r.nmb, on_);
        return on_;
    }
    // frame `fidx`'s records, once analysed (any thread; each frame's slot is its own)
    void record(long long fidx, bool key, const Vp8Mb* mbs, int mb_w, int mb_h) {
        Rec& r = ring_[fidx % kStatsLag];
        r.fidx = fidx;
        r.nmb = mb_w * mb_h;
        r.c = h264::DbAutoCounts{};
        r.valid = !key && mode_ == 2;
        if (!r.valid) return;
        static_assert(sizeof(Vp8Mb) % sizeof(int16_t) == 0, "Vp8Mb: vector words at its start");
        const int16_t* mv = reinterpret_cast<const int16_t*>(mbs);
        for (int i = 0; i < r.nmb; ++i) h264::db_auto_count_mv(mv, (int)(sizeof(Vp8Mb) / sizeof(int16_t)), mb_w, i, r.c);
    }

   private:
    struct Rec {
        long long fidx = -1;
        int nmb = 0;
        bool valid = false;
        h264::DbAutoCounts c;
    };
    int mode_;
    bool on_ = false;
    Rec ring_[kStatsLag];
};

// Small persistent worker pool for the token partitions.
class PartitionPool {
   public:
    explicit PartitionPool(int n);
    ~PartitionPool();
    // Run fn(0 .. n-1) on the pool and the calling thread; several callers (the frame slots'
    // writer threads) may run jobs at once -- their tasks queue in call order on the shared threads.
    void run(int n, const std::function<void(int)>& fn);

   private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int next = 0, total = 0, finished = 0;
    };
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job*> jobs_;  // jobs with tasks not yet taken
    bool stop_ = false;
};

class CpuVp8Encoder {
   public:
    explicit CpuVp8Encoder(const h264::EncoderConfig& cfg);
    const std::vector<uint8_t>& encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr = false);
    const h264::FrameStats& last_stats() const { return stats_; }
    h264::EncoderCommon& common() { return common_; }
    const std::vector<uint8_t>& recon_y() const { return rec_y_[cur_]; }
    const std::vector<uint8_t>& recon_uv() const { return rec_uv_[cur_]; }
    int coded_pitch() const { return cw_; }
    const std::vector<Vp8Mb>& mb_info() const { return mb_; }
    // last frame's bitstream writer time split (host us): first partition, token partitions
    double writer_first_us() const { return tok_stats_[stats_.idr ? 1 : 0][(frames_ - 1) % kStatsLag].us_first; }
    double writer_tokens_us() const { return tok_stats_[stats_.idr ? 1 : 0][(frames_ - 1) % kStatsLag].us_tokens; }

   private:
    void analyse(const uint8_t* y, const uint8_t* uv, int pitch, bool key, int qindex, int qp);
    void intra_pass(const uint8_t* y, const uint8_t* uv, int pitch, int qp);  // inter frames (vp8_core.h)
    h264::EncoderConfig cfg_;
    h264::EncoderCommon common_;
    int cw_, ch_, mb_w_, mb_h_;
    std::vector<uint8_t> rec_y_[2], rec_uv_[2];
    std::vector<uint8_t> prev_src_, next_src_;  // aq >= 3: previous / this frame's source luma (temporal classes)
    // [key][frame % kStatsLag]: branch statistics for the probability updates -- frame n plans
    // from the statistics frame n - kStatsLag left (the GPU encoder writes up to kStatsLag frames
    // concurrently)
    TokenStats tok_stats_[2][kStatsLag];
    long long frames_ = 0;
    int seg_qindex_[kNumSegs] = {0, 0, 0, 0};
    LfDecision lf_;
    int lf_num_ = kLfNumDefault;
    int cur_ = 0;
    bool have_ref_ = false;
    std::vector<Vp8Mb> mb_;
    std::vector<int16_t> lv_;
    std::vector<uint8_t> au_;
    h264::FrameStats stats_;
};

// Device layout of the GPU encoder
constexpr int kKeyLineWords = 8;  // k_vp8_key hand-off words per macroblock
struct Vp8FrameState {
    const uint8_t* ref_y;   // previous reconstruction (P frames)
    const uint8_t* ref_uv;
    uint8_t* rec_y;         // this frame's reconstruction
    uint8_t* rec_uv;
    uint8_t* hp_f;          // padded full-sample reference (origin applied; k_vp8_pad writes it)
    const uint8_t* prev_src;  // aq >= 3: previous frame's source luma (temporal classes; pitch g.pitch)
    uint8_t* save_src;        // aq >= 3: this frame's source luma, kept for the next frame
    int32_t hp_pitch;
    int32_t key;
    int32_t qindex;
    int32_t epoch;          // nonzero, new every frame: tag of the wavefront hand-off words (32 bits)
    int32_t segmented;      // inter frame with segment quantisers (temporal classes)
    int32_t aq;
    int32_t q[kNumSegs][6];   // per segment: Y1 DC, Y1 AC, Y2 DC, Y2 AC, UV DC, UV AC quantiser steps
    uint32_t qm[kNumSegs][6]; // ceil(2^32 / (3 q)): the dead-zone quantiser's division as a multiply-high
    int32_t drop_lambda;    // P frames: lambda_sse of the frame QP for vp8_drop_residual
    int32_t bpred_lambda;   // key frames: lambda_sad of the frame QP for the B_PRED decision (0: no B_PRED)
    int32_t intra_lambda;   // inter frames: lambda_sad of the frame QP for vp8_intra_candidate
    int32_t lf_level[kNumSegs];  // loop-filter level per segment (k_vp8_lf; all 0: not launched)
};
// Both per-frame states in one block: one host->device copy per frame.
struct Vp8States {
    Vp8FrameState v;
    h264::FrameState me;  // motion search state of the shared H.264 kernel (qp, range, planes)
};
struct Vp8DeviceBuffers {
    Vp8States* st;         // device copy of the frame states
    Vp8Mb* mb;             // [nmb] records (device)
    int16_t* lv;           // [nmb * 400] levels (device)
    uint64_t* line;        // [mb_h][mb_w][kKeyLineWords] key-frame hand-off: bottom luma + chroma rows, epoch-tagged
    int* err;              // mapped host word: nonzero if a wavefront spin timed out
    unsigned long long* lf_line;  // loop-filter hand-off lines (k_vp8_lf: epoch-tagged, per workgroup) + scratch
    unsigned long long* lf_sse;  // mapped host [mb_h][3]: Y / U / V distortion of the filtered picture
    Vp8Mb* mb_host;        // mapped host: records with their level slots (k_vp8_gather)
    int16_t* lv_host;      // mapped host: levels of the coded macroblocks, row-compacted
    h264::DeviceBuffers me;  // shared H.264 motion search (fs = &st->me, mb = vectors)
    uint8_t* icand;        // [nmb] inter frames' intra pass: candidate << 7 | best 16x16 mode
    int* ilist;            // [1 + nmb] the intra pass's candidates: count, then macroblock indices
};
// P frames: pad the reference, shared integer motion search, then one wave per macroblock.
// hp_planes: the four padded F / H / V / J planes (h264::launch_hpel) when the motion search refines
// to quarter samples (EncoderConfig::subpel), else hp_planes[0] only (the padded full-sample plane)
void launch_vp8_inter(const h264::Geometry& g, const Vp8DeviceBuffers& b, uint8_t* const hp_planes[4], int hp_pitch,
                      bool subpel, const uint8_t* src_y,
                      const uint8_t* src_uv, hipStream_t stream, bool intra = false);
// Key frames: one wave per macroblock row, rows handing their bottom edges down (wavefront).
void launch_vp8_key(const h264::Geometry& g, const Vp8DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                    hipStream_t stream, bool save_src, bool bpred = false);
// Loop filter of the reconstruction in place (Vp8FrameState::lf_level), its distortion per row.
void launch_vp8_lf(const h264::Geometry& g, const Vp8DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                   hipStream_t stream);
// Records + the coded macroblocks' levels into the mapped host buffers (per-row compaction).
void launch_vp8_gather(const h264::Geometry& g, const Vp8DeviceBuffers& b, hipStream_t stream);

class GpuVp8Encoder final : public VideoEncoder {
   public:
    const char* codec() const override { return "vp8"; }
    static constexpr int kMaxInFlight = kStatsLag;
    GpuVp8Encoder(const h264::EncoderConfig& cfg, hipStream_t stream);
    ~GpuVp8Encoder();
    GpuVp8Encoder(const GpuVp8Encoder&) = delete;
    GpuVp8Encoder& operator=(const GpuVp8Encoder&) = delete;
    const h264::Geometry& geometry() const override { return geom_; }
    int pitch() const override { return geom_.pitch; }
    int depth() const override { return depth_; }
    void submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr = false) override;
    const std::vector<uint8_t>& collect() override;
    const h264::FrameStats& last_stats() const override { return stats_; }
    h264::EncoderCommon& rc() override { return common_; }
    const uint8_t* recon_y() const override { return rec_y_[cur_]; }
    const uint8_t* recon_uv() const override { return rec_uv_[cur_]; }
    hipEvent_t done_event() const override { return last_done_; }
    hipEvent_t pending_done_event() const override { return inflight_.empty() ? last_done_ : slots_[inflight_.front()].done; }
    bool prepare(bool force_idr) override;
    void enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) override;
    void record_start() override;
    void record_done() override;
    h264::EncoderCommon& common() { return common_; }
    // records of the last collected frame (valid until that slot is submitted again)
    const Vp8Mb* last_mb_info() const { return last_mb_; }

   private:
    // Each frame slot has a writer thread: it waits for the slot's GPU work and writes the frame's
    // bitstream at once, so with several frames in flight their bitstreams are written concurrently;
    // collect() only waits for the writer of the oldest.  The writers' token partitions share one
    // pool (pool_), sized to the machine, not one per slot.
    struct Slot {
        Vp8DeviceBuffers buf{};
        Vp8States* st_host = nullptr;  // pinned: copied to buf.st at the start of the frame
        hipEvent_t start = nullptr, done = nullptr;
        bool key = false;
        int qp = 0, qindex = 0;
        bool segmented = false;
        int seg_qindex[kNumSegs] = {0, 0, 0, 0};
        int lf_level[kNumSegs] = {0, 0, 0, 0};  // loop filter (all 0: off)
        bool lf_on = false;
        long long fidx = 0;  // frame index (statistics parity)
        // writer (job / ready under wmu_)
        std::thread writer;
        bool job = false, ready = false, timeout = false;
        std::exception_ptr err;
        std::vector<uint8_t> au;
        uint64_t sse[3] = {0, 0, 0};
        int skipped = 0;
        float ms = 0;
        double wt_us = 0;  // writer time (MXDESK_HOST_TIMING report)
        long long wt_n = 0;
    };
    std::unique_ptr<PartitionPool> pool_;
    void writer_loop(Slot& s);
    void alloc_slot(Slot& s);
    void free_slot(Slot& s);
    void fill_state(Slot& s, bool key, int qp, int ref, int cur);
    int probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp);
    void check_slot(Slot& s);
    void write_slot(const Slot& s, std::vector<uint8_t>& out, bool probe = false);

    h264::EncoderConfig cfg_;
    h264::EncoderCommon common_;
    hipStream_t stream_;
    int depth_ = 1;
    h264::Geometry geom_;
    Slot slots_[kMaxInFlight];
    int next_slot_ = 0, prep_slot_ = 0;
    std::deque<int> inflight_;
    hipEvent_t last_done_ = nullptr;
    const Vp8Mb* last_mb_ = nullptr;
    uint8_t* hp_ = nullptr;  // padded full-sample reference
    uint8_t* hp_sub_[3] = {nullptr, nullptr, nullptr};  // subpel: the padded H / V / J half-sample planes
    int hp_pitch_ = 0;
    uint8_t* rec_y_[2] = {nullptr, nullptr};
    uint8_t* rec_uv_[2] = {nullptr, nullptr};
    uint8_t* src_keep_[2] = {nullptr, nullptr};  // aq >= 3: source luma of the frames in rec_y_[k]
    TokenStats tok_stats_[2][kStatsLag];          // [key][frame % kStatsLag], as CpuVp8Encoder
    LfDecision lf_;
    int lf_num_ = kLfNumDefault;
    long long frames_ = 0;
    int cur_ = 0;
    bool have_ref_ = false;
    uint32_t epoch_ = 0;
    int log2_parts_ = 0;
    int device_ = 0;
    std::mutex wmu_;
    std::condition_variable wcv_;
    bool wstop_ = false;
    std::vector<uint8_t> au_;
    h264::FrameStats stats_;
};

}  // namespace vp8
}  // namespace mx
