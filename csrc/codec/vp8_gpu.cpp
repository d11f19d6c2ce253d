// GpuVp8Encoder: HIP analysis (vp8_kernels.hip) + host boolean coding (vp8_bitstream.cpp).
//
// Per frame, on the caller's stream: one host->device copy of the frame states, the analysis
// kernels (P: pad + shared motion search + k_vp8_inter; key: the k_vp8_key wavefront), then
// k_vp8_gather, which leaves the records and the coded macroblocks' levels in mapped host memory.
// collect() codes the first partition on the calling thread and the token partitions (one per
// group of macroblock rows) on a small worker pool; with pipeline depth 2 that host work overlaps
// the GPU analysis of the next frame.  Decisions and samples equal CpuVp8Encoder's (tests/test_gpu_vp8.py).
#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../common/hip_check.h"
#include "h264_core.h"
#include "h264_mb.h"
#include "vp8_encoder.h"

namespace mx {
namespace vp8 {

namespace {
int pool_threads() {
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::clamp(hc ? hc / 2 : 1u, 1u, 16u);
}
int log2_parts_for(int mb_h) { return mb_h >= 8 ? 3 : (mb_h >= 4 ? 2 : (mb_h >= 2 ? 1 : 0)); }
}  // namespace

void GpuVp8Encoder::alloc_slot(Slot& s) {
    const int nmb = geom_.mb_w * geom_.mb_h;
    Vp8DeviceBuffers& b = s.buf;
    HIP_CHECK(hipMalloc(&b.st, sizeof(Vp8States)));
    HIP_CHECK(hipMalloc(&b.mb, sizeof(Vp8Mb) * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.lv, sizeof(int16_t) * kCoefPerMb * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.line, sizeof(uint64_t) * kKeyLineWords * (size_t)geom_.mb_h * geom_.mb_w));
    HIP_CHECK(hipMemsetAsync(b.line, 0, sizeof(uint64_t) * kKeyLineWords * (size_t)geom_.mb_h * geom_.mb_w, stream_));  // tag 0: no frame
    // hand-off lines: 32 tagged words per macroblock per workgroup of rows, then 1 KB scratch per
    // row (k_vp8_lf); tags start at 0, never a frame's epoch
    const size_t lf_bytes = sizeof(uint64_t) * 32 * (size_t)geom_.mb_h * geom_.mb_w + 1024 * (size_t)(geom_.mb_h + 16);
    HIP_CHECK(hipMalloc(&b.lf_line, lf_bytes));
    HIP_CHECK(hipMemsetAsync(b.lf_line, 0, lf_bytes, stream_));
    HIP_CHECK(hipHostMalloc(&b.lf_sse, sizeof(unsigned long long) * 3 * (size_t)geom_.mb_h, hipHostMallocMapped));
    HIP_CHECK(hipHostMalloc(&b.err, sizeof(int), hipHostMallocMapped));
    *b.err = 0;
    HIP_CHECK(hipHostMalloc(&b.mb_host, sizeof(Vp8Mb) * (size_t)nmb, hipHostMallocMapped));
    HIP_CHECK(hipHostMalloc(&b.lv_host, sizeof(int16_t) * kCoefPerMb * (size_t)nmb, hipHostMallocMapped));
    HIP_CHECK(hipMalloc(&b.me.mb, sizeof(h264::MbInfo) * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.icand, (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.ilist, sizeof(int) * (size_t)(nmb + 1)));
    b.me.fs = &b.st->me;
    HIP_CHECK(hipHostMalloc(&s.st_host, sizeof(Vp8States), hipHostMallocDefault));
    std::memset(s.st_host, 0, sizeof(Vp8States));
    HIP_CHECK(hipEventCreate(&s.start));
    HIP_CHECK(hipEventCreate(&s.done));
}

void GpuVp8Encoder::free_slot(Slot& s) {
    Vp8DeviceBuffers& b = s.buf;
    for (void* p : {(void*)b.st, (void*)b.mb, (void*)b.lv, (void*)b.line, (void*)b.me.mb, (void*)b.lf_line, (void*)b.icand, (void*)b.ilist})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)b.err, (void*)b.mb_host, (void*)b.lv_host, (void*)s.st_host, (void*)b.lf_sse})
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : {s.start, s.done})
        if (e) (void)hipEventDestroy(e);
}

GpuVp8Encoder::GpuVp8Encoder(const h264::EncoderConfig& cfg, hipStream_t stream)
    : cfg_(cfg.with_aq_default(4)),
      common_(cfg),
      stream_(stream),
      lf_(cfg.vp8_deblock_mode()),
      lf_num_(lf_num_from_env()) {
    if (cfg.pipeline_depth < 1 || cfg.pipeline_depth > kMaxInFlight)
        throw std::invalid_argument("pipeline_depth must be 1 to 4");
    if (cfg.width > 16383 || cfg.height > 16383) throw std::invalid_argument("vp8: picture larger than 16383");
    depth_ = cfg.pipeline_depth;
    geom_.width = cfg.width;
    geom_.height = cfg.height;
    geom_.mb_w = common_.mb_w();
    geom_.mb_h = common_.mb_h();
    geom_.coded_w = geom_.mb_w * 16;
    geom_.coded_h = geom_.mb_h * 16;
    geom_.pitch = (geom_.coded_w + 255) & ~255;
    if (geom_.mb_w > 512) throw std::invalid_argument("vp8: picture too wide (k_vp8_gather ranks <= 512 MBs per row)");
    log2_parts_ = log2_parts_for(geom_.mb_h);
    const size_t ysz = (size_t)geom_.pitch * geom_.coded_h, uvsz = ysz / 2;
    for (int i = 0; i < 2; ++i) {
        HIP_CHECK(hipMalloc(&rec_y_[i], ysz));
        HIP_CHECK(hipMalloc(&rec_uv_[i], uvsz));
        HIP_CHECK(hipMemsetAsync(rec_y_[i], 0, ysz, stream_));
        HIP_CHECK(hipMemsetAsync(rec_uv_[i], 128, uvsz, stream_));
        if (cfg_.aq >= 3) {
            HIP_CHECK(hipMalloc(&src_keep_[i], ysz));
            HIP_CHECK(hipMemsetAsync(src_keep_[i], 0, ysz, stream_));
        }
    }
    hp_pitch_ = (geom_.coded_w + 2 * h264::kHpelPad + 255) & ~255;
    HIP_CHECK(hipMalloc(&hp_, (size_t)hp_pitch_ * (geom_.coded_h + 2 * h264::kHpelPad)));
    if (cfg.subpel)
        for (auto& p : hp_sub_) HIP_CHECK(hipMalloc(&p, (size_t)hp_pitch_ * (geom_.coded_h + 2 * h264::kHpelPad)));
    for (int i = 0; i < depth_; ++i) alloc_slot(slots_[i]);
    HIP_CHECK(hipStreamSynchronize(stream_));
    HIP_CHECK(hipGetDevice(&device_));
    // one partition pool for all slot writers (a per-slot pool held up to 36 threads per session at
    // depth 4; a per-slot share of 8 threads cost 40 % of the single-session rate, 7,014 -> 4,413 fps:
    // profiles/r05_vp8/NOTES.md)
    pool_ = std::make_unique<PartitionPool>(pool_threads());
    for (int i = 0; i < depth_; ++i) slots_[i].writer = std::thread([this, i]() { writer_loop(slots_[i]); });
}

void GpuVp8Encoder::writer_loop(Slot& s) {
    (void)hipSetDevice(device_);
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(wmu_);
            wcv_.wait(lk, [&] { return wstop_ || s.job; });
            if (!s.job) return;  // stopping with no frame pending
            s.job = false;
        }
        try {
            HIP_CHECK(hipEventSynchronize(s.done));
            if (*s.buf.err) {  // a key-frame hand-off spin timed out: collect() reports it
                s.timeout = true;
            } else {
                const auto t0 = std::chrono::steady_clock::now();
                s.au.clear();
                write_slot(s, s.au);
                s.wt_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                ++s.wt_n;
                const int nmb = geom_.mb_w * geom_.mb_h;
                s.sse[0] = s.sse[1] = s.sse[2] = 0;
                s.skipped = 0;
                for (int i = 0; i < nmb; ++i) {
                    const Vp8Mb& m = s.buf.mb_host[i];
                    for (int c = 0; c < 3; ++c) s.sse[c] += m.sse[c];
                    s.skipped += m.nz == 0;
                }
                if (s.lf_on) {  // the filtered picture's distortion (k_vp8_lf, per row)
                    s.sse[0] = s.sse[1] = s.sse[2] = 0;
                    for (int r = 0; r < geom_.mb_h; ++r)
                        for (int c = 0; c < 3; ++c) s.sse[c] += s.buf.lf_sse[3 * r + c];
                }
                lf_.record(s.fidx, s.key, s.buf.mb_host, geom_.mb_w, geom_.mb_h);
                s.ms = 0;
                (void)hipEventElapsedTime(&s.ms, s.start, s.done);
            }
        } catch (...) {
            s.err = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> lk(wmu_);
            s.ready = true;
        }
        wcv_.notify_all();
    }
}

GpuVp8Encoder::~GpuVp8Encoder() {
    {
        std::lock_guard<std::mutex> lk(wmu_);
        wstop_ = true;
    }
    wcv_.notify_all();
    double wt_us = 0;
    long long wt_n = 0;
    for (int i = 0; i < depth_; ++i) {
        if (slots_[i].writer.joinable()) slots_[i].writer.join();
        wt_us += slots_[i].wt_us;
        wt_n += slots_[i].wt_n;
    }
    if (wt_n > 0 && std::getenv("MXDESK_HOST_TIMING"))
        std::fprintf(stderr, "[mxdesk] vp8 bitstream writer: %.1f us/frame over %lld frames\n", wt_us / wt_n, wt_n);
    (void)hipStreamSynchronize(stream_);
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(rec_y_[i]);
        (void)hipFree(rec_uv_[i]);
        if (src_keep_[i]) (void)hipFree(src_keep_[i]);
    }
    (void)hipFree(hp_);
    for (auto p : hp_sub_)
        if (p) (void)hipFree(p);
    for (int i = 0; i < depth_; ++i) free_slot(slots_[i]);
}

void GpuVp8Encoder::fill_state(Slot& s, bool key, int qp, int ref, int cur) {
    const size_t org = (size_t)h264::kHpelPad * hp_pitch_ + h264::kHpelPad;
    Vp8FrameState& f = s.st_host->v;
    f.ref_y = rec_y_[ref];
    f.ref_uv = rec_uv_[ref];
    f.rec_y = rec_y_[cur];
    f.rec_uv = rec_uv_[cur];
    f.hp_f = hp_ + org;
    f.hp_pitch = hp_pitch_;
    f.key = key ? 1 : 0;
    s.qindex = qindex_for_qp(qp);
    f.qindex = s.qindex;
    if (++epoch_ == 0) epoch_ = 1;  // 32-bit tag (bits 32..63 of the hand-off words), never 0
    f.epoch = (int32_t)epoch_;
    // inter frames with temporal classes: segment quantisers; key frames: the frame quantiser
    s.segmented = !key && cfg_.aq >= 3;
    for (int k = 0; k < kNumSegs; ++k) s.seg_qindex[k] = s.qindex;
    if (s.segmented) segment_qindices(qp, cfg_.aq, s.seg_qindex);
    f.segmented = s.segmented ? 1 : 0;
    f.aq = cfg_.aq;
    f.prev_src = src_keep_[ref];
    f.save_src = src_keep_[cur];
    for (int k = 0; k < kNumSegs; ++k) {
        const Quant Q = quant_of(s.seg_qindex[k]);
        const int q[6] = {Q.y1dc, Q.y1ac, Q.y2dc, Q.y2ac, Q.uvdc, Q.uvac};
        for (int i = 0; i < 6; ++i) {
            f.q[k][i] = q[i];
            f.qm[k][i] = 0xffffffffu / (uint32_t)(3 * q[i]) + 1u;  // ceil(2^32 / 3q)
        }
    }
    f.drop_lambda = h264::lambda_sse(qp);
    f.bpred_lambda = cfg_.vp8_bpred ? h264::lambda_sad(qp) : 0;
    f.intra_lambda = h264::lambda_sad(qp);
    for (int k = 0; k < kNumSegs; ++k) f.lf_level[k] = s.lf_level[k] = 0;  // prepare() decides the filter
    s.lf_on = false;
    h264::FrameState& m = s.st_host->me;
    std::memset(&m, 0, sizeof m);
    m.ref_y = rec_y_[ref];
    m.ref_uv = rec_uv_[ref];
    m.qp = qp;
    m.search_range = h264::me_range(cfg_.search_range);
    m.me_coarse = cfg_.me_coarse;
    m.subpel = cfg_.subpel ? 1 : 0;  // quarter-sample vectors (VP8 luma precision), six-tap prediction
    m.hp_pitch = hp_pitch_;
    m.hp_f = hp_ + org;
    m.hp_h = (cfg_.subpel ? hp_sub_[0] : hp_) + org;
    m.hp_v = (cfg_.subpel ? hp_sub_[1] : hp_) + org;
    m.hp_j = (cfg_.subpel ? hp_sub_[2] : hp_) + org;
}

void GpuVp8Encoder::enqueue_body(bool key, const uint8_t* src_y, const uint8_t* src_uv) {
    Slot& s = slots_[prep_slot_];
    HIP_CHECK(hipMemcpyAsync(s.buf.st, s.st_host, sizeof(Vp8States), hipMemcpyHostToDevice, stream_));
    if (key)
        launch_vp8_key(geom_, s.buf, src_y, src_uv, stream_, cfg_.aq >= 3, cfg_.vp8_bpred != 0);
    else
    {
        uint8_t* const planes[4] = {hp_, hp_sub_[0], hp_sub_[1], hp_sub_[2]};
        launch_vp8_inter(geom_, s.buf, planes, hp_pitch_, cfg_.subpel != 0, src_y, src_uv, stream_, cfg_.vp8_intra != 0);
    }
    if (s.lf_on) launch_vp8_lf(geom_, s.buf, src_y, src_uv, stream_);
    launch_vp8_gather(geom_, s.buf, stream_);
    HIP_CHECK(hipGetLastError());
}

void GpuVp8Encoder::check_slot(Slot& s) {
    if (*s.buf.err) {  // a key-frame hand-off spin timed out: the reconstruction is unreliable
        *s.buf.err = 0;
        have_ref_ = false;
        throw std::runtime_error("vp8 gpu encoder: key-frame wavefront hand-off timed out");
    }
}

void GpuVp8Encoder::write_slot(const Slot& s, std::vector<uint8_t>& out, bool probe) {
    const Vp8Mb* mbs = s.buf.mb_host;
    const int16_t* lv = s.buf.lv_host;
    FrameDesc fd{s.key, cfg_.width, cfg_.height, geom_.mb_w, geom_.mb_h, s.qindex, log2_parts_};
    fd.segmented = s.segmented;
    for (int k = 0; k < kNumSegs; ++k) {
        fd.seg_qindex[k] = s.seg_qindex[k];
        fd.lf_level[k] = s.lf_level[k];
    }
    // k_vp8_gather sent only the blocks with a non-zero level (16 levels each, from block `slot`):
    // expanded into the 25-block layout the token writer reads, one macroblock at a time per thread
    auto levels = [&](int i) -> const int16_t* {
        thread_local int16_t full[kCoefPerMb];
        const Vp8Mb& m = mbs[i];
        const int16_t* p = lv + (size_t)m.slot * 16;
        for (int b = 0; b < kBlocks; ++b) {
            if ((m.nz >> b) & 1u) {
                std::memcpy(full + b * 16, p, 16 * sizeof(int16_t));
                p += 16;
            } else {
                std::memset(full + b * 16, 0, 16 * sizeof(int16_t));
            }
        }
        return full;
    };
    write_frame(fd, mbs, levels, out,
                [&](int n, const std::function<void(int)>& fn) { pool_->run(n, fn); },
                probe ? nullptr : &tok_stats_[s.key ? 1 : 0][s.fidx % kStatsLag]);
}

int GpuVp8Encoder::probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp) {
    // synchronous key frame at `qp` (the rate controller's first-frame probe); the real first
    // frame overwrites the reconstruction
    if (!inflight_.empty()) throw std::logic_error("GpuVp8Encoder: probe with frames in flight");
    prep_slot_ = 0;
    Slot& s = slots_[0];
    s.key = true;
    fill_state(s, true, qp, cur_ ^ 1, cur_);
    enqueue_body(true, src_y, src_uv);
    HIP_CHECK(hipStreamSynchronize(stream_));
    check_slot(s);
    std::vector<uint8_t> tmp;
    write_slot(s, tmp, true);
    return (int)tmp.size();
}

bool GpuVp8Encoder::prepare(bool force_idr) {
    if ((int)inflight_.size() >= depth_) throw std::logic_error("GpuVp8Encoder: collect() a frame first (pipeline full)");
    const int n = (depth_ == 1) ? 0 : next_slot_;
    next_slot_ = (next_slot_ + 1) % depth_;
    prep_slot_ = n;
    Slot& s = slots_[n];
    common_.begin_frame(force_idr || !have_ref_);
    have_ref_ = true;
    s.key = common_.cur_idr();
    s.qp = common_.cur_qp();
    s.fidx = frames_++;
    const int ref = cur_;
    cur_ ^= 1;
    fill_state(s, s.key, s.qp, ref, cur_);
    lf_levels(lf_.decide(s.fidx, s.key), s.segmented, s.qindex, s.seg_qindex, lf_num_, s.lf_level);
    for (int k = 0; k < kNumSegs; ++k) {
        s.st_host->v.lf_level[k] = s.lf_level[k];
        s.lf_on = s.lf_on || s.lf_level[k] != 0;
    }
    return s.key;
}

void GpuVp8Encoder::record_start() { HIP_CHECK(hipEventRecord(slots_[prep_slot_].start, stream_)); }

void GpuVp8Encoder::record_done() {
    Slot& s = slots_[prep_slot_];
    HIP_CHECK(hipEventRecord(s.done, stream_));
    inflight_.push_back(prep_slot_);
    {
        std::lock_guard<std::mutex> lk(wmu_);
        s.job = true;
        s.ready = false;
    }
    wcv_.notify_all();
}

void GpuVp8Encoder::submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr) {
    while (common_.wants_probe()) {
        const int q = common_.probe_qp();
        common_.add_probe(q, probe_bytes(src_y, src_uv, q));
    }
    const bool key = prepare(force_idr);
    record_start();
    enqueue_body(key, src_y, src_uv);
    record_done();
}

const std::vector<uint8_t>& GpuVp8Encoder::collect() {
    if (inflight_.empty()) throw std::logic_error("GpuVp8Encoder: nothing submitted");
    const int n = inflight_.front();
    inflight_.pop_front();
    Slot& s = slots_[n];
    {
        std::unique_lock<std::mutex> lk(wmu_);
        wcv_.wait(lk, [&] { return s.ready; });
        s.ready = false;
    }
    last_done_ = s.done;
    last_mb_ = s.buf.mb_host;
    if (s.timeout || s.err) {
        std::exception_ptr e = s.err;
        s.err = nullptr;
        const bool timeout = s.timeout;
        s.timeout = false;
        common_.end_frame(0, s.key);
        if (timeout) check_slot(s);  // clears the error word, drops the reference, throws
        std::rethrow_exception(e);
    }
    au_.swap(s.au);
    stats_.frame_index = common_.frames();
    stats_.idr = s.key;
    stats_.qp = s.qp;
    stats_.bytes = (int)au_.size();
    stats_.encode_ms = s.ms;
    stats_.skipped_mbs = s.skipped;
    stats_.deblocked = s.lf_on;
    for (int c = 0; c < 3; ++c) stats_.sse[c] = s.sse[c];
    stats_.sse_masked = s.sse[0];
    stats_.masked_pixels = (int64_t)cfg_.width * cfg_.height;
    common_.end_frame((int)au_.size(), s.key);
    return au_;
}

}  // namespace vp8
}  // namespace mx
