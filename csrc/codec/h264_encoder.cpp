// Host driver of the HIP H.264 encoder + the Annex-B / rate-control logic shared with
// the CPU encoder.  See h264_gpu.h for the kernel chain.
#include "h264_encoder.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../common/hip_check.h"
#include "h264_mb.h"

namespace mx {
namespace h264 {

// ------------------------------------------------------------------ EncoderCommon
EncoderCommon::EncoderCommon(const EncoderConfig& c) : cfg_(c) {
    if (c.width <= 0 || c.height <= 0 || (c.width & 1) || (c.height & 1))
        throw std::invalid_argument("encoder size must be positive and even");
    mb_w_ = (c.width + 15) / 16;
    mb_h_ = (c.height + 15) / 16;
    cur_qp_ = std::clamp(c.qp, 0, 51);
}

double EncoderCommon::frame_budget_bits() const {
    return cfg_.bitrate_kbps * 1000.0 / std::max(1, cfg_.fps);
}

int EncoderCommon::qp_for(double x, double bits, double alpha) const {
    // bits = x / qstep(qp)^alpha  =>  qp = 6 * log2((x / bits)^(1/alpha) / 0.625)
    const double r = std::max(1e-9, x) / std::max(1.0, bits);
    const double q = 6.0 * std::log2(std::pow(r, 1.0 / alpha) / 0.625);
    return (int)std::lround(std::clamp(q, 0.0, 51.0));
}

int EncoderCommon::probe_qp() const {
    if (probes_ == 0) {
        // prior: ~1 bit per luma sample at QP 30 for desktop content, scaled to the IDR budget
        const double px = (double)cfg_.width * cfg_.height;
        return std::clamp(qp_for(px * qstep(30), kIdrBudget * frame_budget_bits(), 1.0), cfg_.qp_min, cfg_.qp_max);
    }
    return std::clamp(qp_for(x_i_, kIdrBudget * frame_budget_bits(), 1.0), cfg_.qp_min, cfg_.qp_max);
}

void EncoderCommon::add_probe(int qp, int bytes) {
    probe_q_[probes_ < kMaxProbes ? probes_ : kMaxProbes - 1] = qp;
    ++probes_;
    x_i_ = std::max(8.0, bytes * 8.0) * qstep(qp);
    // a second probe only if the first one was far from the budget
    const int next = probe_qp();
    if (probes_ >= kMaxProbes || std::abs(next - qp) <= 2) probe_done_ = true;
}

void EncoderCommon::begin_frame(bool force_idr) {
    // frame counters advance here (not in end_frame) so that a second frame can be begun
    // before the first one is finished (pipelined GPU encode)
    const bool idr = idr_requested_ || force_idr || begun_ == 0 || (cfg_.keyint > 0 && since_idr_ >= cfg_.keyint);
    cur_idr_ = idr;
    idr_requested_ = false;
    ++begun_;
    probe_done_ = true;  // probing only ever precedes the first frame
    if (idr) {
        frame_num_ = 0;
        idr_pic_id_ = (idr_pic_id_ + 1) & 0xffff;
        since_idr_ = 1;
    } else {
        frame_num_ = (frame_num_ + 1) % (1 << log2_max_frame_num());
        ++since_idr_;
    }
    if (cfg_.bitrate_kbps <= 0) {
        cur_qp_ = std::clamp(cfg_.qp, 0, 51);
        return;
    }
    const double T = frame_budget_bits();
    // buffer state including the frames still in flight, charged at their budgets
    double vbv = vbv_;
    for (const Pending& p : pending_) vbv += p.budget - T;
    double budget;
    int q;
    if (idr) {
        budget = kIdrBudget * T;
        const double x = x_i_ > 0 ? x_i_ : (double)cfg_.width * cfg_.height * qstep(30);
        q = qp_for(x, budget, 1.0);
    } else {
        // linear drain of the buffer excess over the recovery window that follows an IDR
        // (the whole excess is paid back kDrainFrames after it), then a gentle correction
        const int64_t k = since_idr_ - 1;  // P frames since the IDR, this one included
        const double div = k <= kDrainFrames ? (double)(kDrainFrames - k + 1) : 3.0;
        budget = std::clamp(T - vbv / div, 0.25 * T, 2.0 * T);
        if (x_p_ > 0) {
            q = qp_for(x_p_, budget, alpha_p_);
        } else if (x_i_ > 0) {
            // no P picture finished yet: assume a P picture costs kPPrior of an I picture at equal
            // QP (desktop P pictures cost 10-20 % of the IDR; the former 0.5 starved the first P
            // pictures at QP 46 after every IDR; the model has real P data two frames later)
            q = qp_for(kPPrior * x_i_, budget, 1.0);
        } else {
            q = (last_i_qp_ >= 0 ? last_i_qp_ : cfg_.qp) + 2;
        }
        // asymmetric step limits: lowering the QP below the reference's makes the picture
        // refine the whole reference (a P at QP-3 after a coarse IDR cost 2.6 budgets on the
        // 1080p desktop: profiles/r02_rc), so QP falls by at most kMaxDown per frame; rising is
        // cheap and protects the buffer.  Right after an IDR the ramp starts from the IDR's QP.
        if (last_was_idr_)
            q = std::max(q, last_p_qp_ - kMaxDown);
        else if (last_p_qp_ >= 0)
            q = std::clamp(q, last_p_qp_ - kMaxDown, last_p_qp_ + kMaxStep);
    }
    cur_qp_ = std::clamp(std::clamp(q, cfg_.qp_min, cfg_.qp_max), 0, 51);
    pending_.push_back(Pending{budget, cur_qp_, idr, since_idr_});
    last_p_qp_ = cur_qp_;  // an IDR anchors the next P: its QP ramps down from the IDR's by
                           // kMaxStep per frame instead of refining the whole picture at once
    if (idr) last_i_qp_ = cur_qp_;
    last_was_idr_ = idr;
}

void EncoderCommon::end_frame(int bytes, bool idr) {
    ++frame_index_;
    if (pending_.empty()) return;  // constant QP (nothing tracked)
    const Pending p = pending_.front();
    pending_.pop_front();
    if (cfg_.bitrate_kbps <= 0) return;
    const double T = frame_budget_bits();
    const double bits = bytes * 8.0;
    vbv_ = std::max(-2.0 * T, vbv_ + bits - T);
    const double b = std::max(8.0, bits);
    if (idr || p.idr) {
        x_i_ = b * qstep(p.qp);
        return;
    }
    // local slope of the rate-QP curve from consecutive P pictures at different QPs (desktop
    // content is far from bits ~ 1/qstep: adaptive quantisation saturates noise-like areas)
    // (not across the refinement frames right after an IDR: their cost reflects the IDR's
    // quality, not the content's rate-QP slope)
    if (prev_p_bits_ > 0 && prev_p_qp_ != p.qp && p.since_idr > kDrainFrames / 2) {
        const double a = std::log(prev_p_bits_ / b) / std::log(qstep(p.qp) / qstep(prev_p_qp_));
        alpha_p_ = 0.5 * alpha_p_ + 0.5 * std::clamp(a, 0.6, 3.0);
    }
    prev_p_bits_ = b;
    prev_p_qp_ = p.qp;
    x_p_ = b * std::pow(qstep(p.qp), alpha_p_);
}

static void words_to_bytes(const uint32_t* w, uint32_t bits, std::vector<uint8_t>& out) {
    const uint32_t nbytes = (bits + 7) / 8;
    for (uint32_t i = 0; i < nbytes; ++i) out.push_back((uint8_t)(w[i / 4] >> (24 - 8 * (i % 4))));
}

void emulation_prevent(std::vector<uint8_t>& out, const uint8_t* rbsp, size_t n) {
    int zeros = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t b = rbsp[i];
        if (zeros >= 2 && b <= 3) {
            out.push_back(3);
            zeros = 0;
        }
        out.push_back(b);
        zeros = (b == 0) ? zeros + 1 : 0;
    }
}

void EncoderCommon::write_parameter_sets(std::vector<uint8_t>& out) const {
    uint32_t words[64];
    SeqParams sp;
    sp.width = cfg_.width;
    sp.height = cfg_.height;
    sp.mb_w = mb_w_;
    sp.mb_h = mb_h_;
    sp.level_idc = pick_level(mb_w_ * mb_h_, cfg_.fps);
    sp.log2_max_frame_num = log2_max_frame_num();
    sp.fps_num = cfg_.fps;
    sp.fps_den = 1;
    BitWriter w;
    w.init(words);
    write_sps(w, sp);
    std::vector<uint8_t> rbsp;
    words_to_bytes(words, w.bits + (w.bits % 8 ? 8 - w.bits % 8 : 0), rbsp);
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back(0x67);  // nal_ref_idc 3, SPS
    emulation_prevent(out, rbsp.data(), rbsp.size());
    w.init(words);
    write_pps(w, pic_init_qp(), cfg_.chroma_qp_offset);
    rbsp.clear();
    words_to_bytes(words, w.bits + (w.bits % 8 ? 8 - w.bits % 8 : 0), rbsp);
    out.insert(out.end(), sc, sc + 4);
    out.push_back(0x68);  // PPS
    emulation_prevent(out, rbsp.data(), rbsp.size());
}

void EncoderCommon::write_slice_nal(std::vector<uint8_t>& out, const uint8_t* rbsp, size_t n, bool idr) const {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back(idr ? 0x65 : 0x41);  // IDR slice (ref_idc 3) / non-IDR slice (ref_idc 2)
    emulation_prevent(out, rbsp, n);
}

// ------------------------------------------------------------------ test hook: half-sample planes
std::vector<std::vector<uint8_t>> hpel_planes_for_test(const uint8_t* ref, int coded_w, int coded_h, int pitch,
                                                       int* hp_pitch_out) {
    Geometry g{};
    g.width = coded_w;
    g.height = coded_h;
    g.mb_w = coded_w / 16;
    g.mb_h = coded_h / 16;
    g.coded_w = coded_w;
    g.coded_h = coded_h;
    g.pitch = pitch;
    const int hp_pitch = (coded_w + 2 * kHpelPad + 255) & ~255;
    const size_t hp_bytes = (size_t)hp_pitch * (coded_h + 2 * kHpelPad);
    uint8_t* dref = nullptr;
    uint8_t* planes[4];
    FrameState fs{};
    DeviceBuffers b{};
    HIP_CHECK(hipMalloc(&dref, (size_t)pitch * coded_h));
    HIP_CHECK(hipMemcpy(dref, ref, (size_t)pitch * coded_h, hipMemcpyHostToDevice));
    for (auto& p : planes) {
        HIP_CHECK(hipMalloc(&p, hp_bytes));
        HIP_CHECK(hipMemset(p, 0, hp_bytes));
    }
    fs.ref_y = dref;
    HIP_CHECK(hipMalloc(&b.fs, sizeof(FrameState)));
    HIP_CHECK(hipMemcpy(b.fs, &fs, sizeof(FrameState), hipMemcpyHostToDevice));
    launch_hpel(g, b, planes, hp_pitch, nullptr);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
    std::vector<std::vector<uint8_t>> out(4, std::vector<uint8_t>(hp_bytes));
    for (int i = 0; i < 4; ++i) {
        HIP_CHECK(hipMemcpy(out[i].data(), planes[i], hp_bytes, hipMemcpyDeviceToHost));
        (void)hipFree(planes[i]);
    }
    (void)hipFree(dref);
    (void)hipFree(b.fs);
    *hp_pitch_out = hp_pitch;
    return out;
}

// ------------------------------------------------------------------ GpuH264Encoder
// Events that only order GPU work between this device's queues: a device-scope release when
// recorded (the default system-scope release writes the caches back for the host each time).
constexpr unsigned kDeviceEvent = hipEventDisableTiming | hipEventReleaseToDevice;

void GpuH264Encoder::alloc_slot(FrameSlot& sl) {
    const int nmb = geom_.mb_w * geom_.mb_h;
    DeviceBuffers& b = sl.buf;
    HIP_CHECK(hipMalloc(&b.fs, sizeof(FrameState)));
    HIP_CHECK(hipMalloc(&b.mb, sizeof(MbInfo) * nmb));
    HIP_CHECK(hipMemsetAsync(b.mb, 0, sizeof(MbInfo) * nmb, stream_));
    HIP_CHECK(hipMalloc(&b.coef, sizeof(int16_t) * kCoefStride * nmb));
    HIP_CHECK(hipMalloc(&b.slot, sizeof(uint32_t) * kSlotWords * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.slot_bits, sizeof(uint32_t) * nmb));
    HIP_CHECK(hipMalloc(&b.row_agg, sizeof(uint4) * (size_t)geom_.mb_h));
    HIP_CHECK(hipMalloc(&b.row_sse, sizeof(unsigned long long) * 4 * 512));
    HIP_CHECK(hipMalloc(&b.coded_info, sizeof(uint4) * nmb));
    HIP_CHECK(hipMalloc(&b.slice_info, sizeof(uint32_t) * kSliceInfo * kMaxSlices));
    HIP_CHECK(hipMemsetAsync(b.slice_info, 0, sizeof(uint32_t) * kSliceInfo * kMaxSlices, stream_));
    // payload capacity: 768 B per MB (intra at low QP stays far below)
    b.out_bytes = (size_t)nmb * 768;
    HIP_CHECK(hipMalloc(&b.quad_unit, sizeof(uint32_t) * (b.out_bytes / 16 + 1)));
    HIP_CHECK(hipMalloc(&b.out_hdr, sizeof(OutHeader)));
    HIP_CHECK(hipMalloc(&b.sse_part, 4 * sizeof(unsigned long long) * kSsePartStride));
    HIP_CHECK(hipMalloc(&b.wave_prog, sizeof(int) * 4));
    HIP_CHECK(hipMalloc(&b.mb_sse, sizeof(uint32_t) * 3 * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.intra_gain, sizeof(int32_t) * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.intra_cand, sizeof(int) * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.db_rec, sizeof(uint4) * (size_t)nmb));
    HIP_CHECK(hipMalloc(&b.db_rowq, sizeof(int) * (size_t)geom_.mb_h));
    HIP_CHECK(hipMalloc(&b.db_glb, sizeof(uint64_t) * 2 * 24 * (size_t)nmb));
    HIP_CHECK(hipMemsetAsync(b.db_glb, 0, sizeof(uint64_t) * 2 * 24 * (size_t)nmb, stream_));  // tag 0: no frame
    HIP_CHECK(hipMalloc(&b.pack_done, sizeof(uint32_t)));
    HIP_CHECK(hipMemsetAsync(b.pack_done, 0, sizeof(uint32_t), stream_));
    HIP_CHECK(hipMalloc(&b.db_cnt, sizeof(uint32_t) * 4));
    HIP_CHECK(hipMemsetAsync(b.db_cnt, 0, sizeof(uint32_t) * 4, stream_));
    HIP_CHECK(hipHostMalloc(&b.db_err, sizeof(int), hipHostMallocMapped));
    *b.db_err = 0;
    HIP_CHECK(hipHostMalloc(&sl.fs_host, sizeof(FrameState), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc(&sl.host_out, kOutPayloadOffset + b.out_bytes + 16, hipHostMallocMapped));
    std::memset(sl.host_out, 0, kOutPayloadOffset);
    HIP_CHECK(hipEventCreateWithFlags(&sl.start, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&sl.analysis_done, kDeviceEvent));
    HIP_CHECK(hipEventCreateWithFlags(&sl.deblock_done, kDeviceEvent));
    HIP_CHECK(hipEventCreateWithFlags(&sl.hpel_done, kDeviceEvent));
    HIP_CHECK(hipEventCreateWithFlags(&sl.me_done, kDeviceEvent));
    HIP_CHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
}

void GpuH264Encoder::free_slot(FrameSlot& sl) {
    DeviceBuffers& b = sl.buf;
    for (void* p : {(void*)b.fs, (void*)b.mb, (void*)b.coef, (void*)b.slot, (void*)b.slot_bits, (void*)b.row_agg,
                    (void*)b.row_sse, (void*)b.coded_info, (void*)b.slice_info,
                    (void*)b.out_hdr, (void*)b.sse_part, (void*)b.wave_prog, (void*)b.mb_sse, (void*)b.intra_gain, (void*)b.intra_cand, (void*)b.quad_unit,
                    (void*)b.db_rec, (void*)b.db_rowq, (void*)b.db_glb, (void*)b.pack_done, (void*)b.db_cnt})
        if (p) (void)hipFree(p);
    if (b.db_err) (void)hipHostFree(b.db_err);
    if (sl.fs_host) (void)hipHostFree(sl.fs_host);
    if (sl.host_out) (void)hipHostFree(sl.host_out);
    for (hipEvent_t e : {sl.start, sl.analysis_done, sl.deblock_done, sl.done, sl.hpel_done, sl.me_done})
        if (e) (void)hipEventDestroy(e);
}

GpuH264Encoder::GpuH264Encoder(const EncoderConfig& cfg, hipStream_t stream)
    : cfg_(cfg.with_aq_default(4)), common_(cfg), stream_(stream) {
    if (cfg.pipeline_depth < 1 || cfg.pipeline_depth > kMaxInFlight)
        throw std::invalid_argument("pipeline_depth must be 1 to 4");
    depth_ = cfg.pipeline_depth;
    db_lag_.reset(cfg_.h264_deblock_mode());
    geom_.width = cfg.width;
    geom_.height = cfg.height;
    geom_.mb_w = common_.mb_w();
    geom_.mb_h = common_.mb_h();
    geom_.coded_w = geom_.mb_w * 16;
    geom_.coded_h = geom_.mb_h * 16;
    geom_.pitch = (geom_.coded_w + 255) & ~255;
    if (geom_.mb_h > kMaxSlices) throw std::invalid_argument("picture too tall");
    if (geom_.mb_w > 512) throw std::invalid_argument("picture too wide (k_intra_wave stages <= 512 MBs per row)");
    const int nmb = geom_.mb_w * geom_.mb_h;
    if ((nmb + 3) / 4 + geom_.mb_h > kSsePartStride)
        throw std::invalid_argument("frame too large for the distortion partials");
    const size_t ysz = (size_t)geom_.pitch * geom_.coded_h, uvsz = ysz / 2;
    for (int i = 0; i < 2; ++i) {
        HIP_CHECK(hipMalloc(&rec_y_[i], ysz));
        HIP_CHECK(hipMalloc(&rec_uv_[i], uvsz));
        HIP_CHECK(hipMemsetAsync(rec_y_[i], 16, ysz, stream_));
        HIP_CHECK(hipMemsetAsync(rec_uv_[i], 128, uvsz, stream_));
        HIP_CHECK(hipMalloc(&src_keep_[i], ysz));
        HIP_CHECK(hipMemsetAsync(src_keep_[i], 16, ysz, stream_));
    }
    if (cfg.mask_x1 > cfg.mask_x0 && cfg.mask_y1 > cfg.mask_y0) {
        mask_mb_[0] = std::max(0, cfg.mask_x0) / 16;
        mask_mb_[1] = std::max(0, cfg.mask_y0) / 16;
        mask_mb_[2] = std::min(geom_.mb_w, (cfg.mask_x1 + 15) / 16);
        mask_mb_[3] = std::min(geom_.mb_h, (cfg.mask_y1 + 15) / 16);
    }
    masked_pixels_ = (int64_t)cfg.width * cfg.height;
    for (int my = mask_mb_[1]; my < mask_mb_[3]; ++my)
        for (int mx = mask_mb_[0]; mx < mask_mb_[2]; ++mx)
            masked_pixels_ -= (int64_t)std::max(0, std::min(16, cfg.width - 16 * mx)) *
                              std::max(0, std::min(16, cfg.height - 16 * my));
    hp_pitch_ = (geom_.coded_w + 2 * kHpelPad + 255) & ~255;
    const size_t hp_bytes = (size_t)hp_pitch_ * (geom_.coded_h + 2 * kHpelPad);
    for (int i = 0; i < 4; ++i) HIP_CHECK(hipMalloc(&hp_[i], hp_bytes));
    if (cfg_.h264_deblock())
        for (int i = 0; i < 4; ++i) HIP_CHECK(hipMalloc(&hpu_[i], hp_bytes));
    for (int i = 0; i < depth_; ++i) alloc_slot(slots_[i]);
    clock_khz_ = device_clock_khz();
    if (depth_ > 1) {
        HIP_CHECK(hipStreamCreateWithFlags(&stream_e_, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&stream_a_, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&ref_ready_, kDeviceEvent));
        HIP_CHECK(hipEventRecord(ref_ready_, stream_));
        if (cfg_.h264_deblock()) {
            // The side-stream search may keep every CU busy just as the previous picture's
            // k_deblock starts: MXDESK_ME_CU_RESERVE=n (default 0) keeps the search off n compute
            // units (a CU mask on its stream), so the filter's row waves find CUs of their own
            const char* rv = std::getenv("MXDESK_ME_CU_RESERVE");
            const int reserve = rv ? std::atoi(rv) : 0;
            int ncu = 0;
            HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
            if (reserve > 0 && reserve < ncu) {
                std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
                for (int c = 0; c < ncu - reserve; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
                HIP_CHECK(hipExtStreamCreateWithCUMask(&stream_m_, (uint32_t)mask.size(), mask.data()));
            } else {
                HIP_CHECK(hipStreamCreateWithFlags(&stream_m_, hipStreamNonBlocking));
            }
            HIP_CHECK(hipEventCreateWithFlags(&ev_hpu_, kDeviceEvent));
            HIP_CHECK(hipEventRecord(ev_hpu_, stream_));
        }
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
    const char* et = std::getenv("MXDESK_ENTROPY_THREAD");
    if (stream_e_ && !(et && et[0] == '0')) {
        HIP_CHECK(hipGetDevice(&device_));
        launcher_ = std::thread([this]() { launcher_loop(); });
    }
}

void GpuH264Encoder::set_hpel_side_stream(bool on) {
    hpel_side_ = on;
    if (!on && stream_a_) {  // its hardware queue is better left to the session's other streams
        HIP_CHECK(hipStreamSynchronize(stream_a_));
        HIP_CHECK(hipStreamDestroy(stream_a_));
        stream_a_ = nullptr;
    }
}

void GpuH264Encoder::launcher_loop() {
    (void)hipSetDevice(device_);
    for (;;) {
        EntropyJob j;
        {
            std::unique_lock<std::mutex> lk(lmu_);
            lcv_.wait(lk, [&] { return lstop_ || !ljobs_.empty(); });
            if (ljobs_.empty()) return;  // stopping, nothing pending
            j = ljobs_.front();
            ljobs_.pop_front();
        }
        try {
            FrameSlot& sl = slots_[j.slot];
            HIP_CHECK(hipStreamWaitEvent(stream_e_, sl.analysis_done, 0));
            launch_entropy(geom_, sl.buf, sl.host_out, stream_e_, j.sse_ready);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipEventRecord(sl.done, stream_e_));
        } catch (...) {
            std::lock_guard<std::mutex> lk(lmu_);
            lerr_ = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> lk(lmu_);
            ++l_done_;
        }
        lcv_.notify_all();
    }
}

void GpuH264Encoder::drain_launcher() const {
    // graph capture / replay issues entropy-stream work from this thread: the launcher's queued
    // eager frames go first (and none of its operations may land inside a capture)
    if (!launcher_.joinable()) return;
    std::unique_lock<std::mutex> lk(lmu_);
    lcv_.wait(lk, [&] { return l_done_ >= l_pushed_ || lerr_; });
    if (lerr_) std::rethrow_exception(lerr_);
}

void GpuH264Encoder::wait_launched(int slot) const {
    std::unique_lock<std::mutex> lk(lmu_);
    lcv_.wait(lk, [&] { return l_done_ >= slot_job_[slot] || lerr_; });
    if (lerr_) std::rethrow_exception(lerr_);
}

GpuH264Encoder::~GpuH264Encoder() {
    if (launcher_.joinable()) {  // issues what is queued, then exits
        {
            std::lock_guard<std::mutex> lk(lmu_);
            lstop_ = true;
        }
        lcv_.notify_all();
        launcher_.join();
    }
    (void)hipStreamSynchronize(stream_);
    if (stream_e_) {
        (void)hipStreamSynchronize(stream_e_);
        (void)hipStreamDestroy(stream_e_);
    }
    if (stream_a_) {
        (void)hipStreamSynchronize(stream_a_);
        (void)hipStreamDestroy(stream_a_);
    }
    if (ref_ready_) (void)hipEventDestroy(ref_ready_);
    if (stream_m_) {
        (void)hipStreamSynchronize(stream_m_);
        (void)hipStreamDestroy(stream_m_);
    }
    if (ev_hpu_) (void)hipEventDestroy(ev_hpu_);
    for (int i = 0; i < 4; ++i)
        if (hpu_[i]) (void)hipFree(hpu_[i]);
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(rec_y_[i]);
        (void)hipFree(rec_uv_[i]);
        (void)hipFree(src_keep_[i]);
    }
    for (int i = 0; i < 4; ++i) (void)hipFree(hp_[i]);
    for (int i = 0; i < depth_; ++i) free_slot(slots_[i]);
}

void GpuH264Encoder::enqueue_analysis_kernels(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish) {
    FrameSlot& sl = slots_[prep_slot_];
    const FrameState* pub = publish ? sl.fs_host : nullptr;
    auto wait_input = [&]() {
        if (!in_ev_) return;
        HIP_CHECK(hipStreamWaitEvent(stream_, in_ev_, 0));
        in_ev_ = nullptr;
    };
    if (idr) {
        wait_input();
        launch_intra(geom_, sl.buf, src_y, src_uv, stream_, pub);
        if (cfg_.aq >= 3)  // the next P picture's previous source (P pictures: k_inter_encode stores it)
            launch_save_src(geom_, sl.buf, src_y, stream_);
    } else {
        // MXDESK_INPUT_WAIT=early: the capture hand-off waited before k_hpel (next to the previous
        // frame's analysis_done record) instead of after it -- experiment on queue barrier costs
        static const bool early = [] {
            const char* e = std::getenv("MXDESK_INPUT_WAIT");
            return e && std::string(e) == "early";
        }();
        if (early) wait_input();
        // the search of a picture whose reference was deblocked reads that reference's unfiltered
        // planes (hpu_): on the side stream, it overlaps the reference's k_deblock
        const bool side_me = stream_m_ && pub && sl.me_unf;
        if (side_me) {
            HIP_CHECK(hipStreamWaitEvent(stream_m_, ev_hpu_, 0));
            if (in_ev_) {
                HIP_CHECK(hipStreamWaitEvent(stream_m_, in_ev_, 0));
                in_ev_ = nullptr;  // the analysis stream waits for the search, so for the input too
            }
            launch_me(geom_, sl.buf, src_y, stream_m_, pub);
            HIP_CHECK(hipEventRecord(sl.me_done, stream_m_));
        }
        if (stream_a_ && hpel_side_ && pub && ref_seq_ + 1 == seq_) {  // the previous picture recorded ref_ready_
            HIP_CHECK(hipStreamWaitEvent(stream_a_, ref_ready_, 0));
            launch_hpel(geom_, sl.buf, hp_, hp_pitch_, stream_a_, pub);
            HIP_CHECK(hipEventRecord(sl.hpel_done, stream_a_));
            HIP_CHECK(hipStreamWaitEvent(stream_, sl.hpel_done, 0));
        } else {
            launch_hpel(geom_, sl.buf, hp_, hp_pitch_, stream_, pub);
        }
        wait_input();
        if (side_me)
            HIP_CHECK(hipStreamWaitEvent(stream_, sl.me_done, 0));
        else
            launch_me(geom_, sl.buf, src_y, stream_);
        launch_inter(geom_, sl.buf, src_y, src_uv, stream_);
        if (cfg_.intra_in_p) launch_intra_in_p(geom_, sl.buf, src_y, src_uv, stream_);
    }
}

void GpuH264Encoder::link_entropy() {
    if (!stream_e_) return;
    drain_launcher();  // entropy of this frame overlaps the analysis of the next one
    FrameSlot& sl = slots_[prep_slot_];
    HIP_CHECK(hipEventRecord(sl.analysis_done, stream_));
    HIP_CHECK(hipStreamWaitEvent(stream_e_, sl.analysis_done, 0));
}

void GpuH264Encoder::enqueue_entropy() {
    drain_launcher();
    FrameSlot& sl = slots_[prep_slot_];
    launch_entropy(geom_, sl.buf, sl.host_out, stream_e_ ? stream_e_ : stream_, nullptr);
}

void GpuH264Encoder::unfiltered_planes(FrameSlot& sl) {
    // F/H/V/J planes of this picture's reconstruction before k_deblock filters it in place: the
    // next picture's motion search (FrameState::me_*) reads them on the side stream
    launch_hpel_of(geom_, sl.fs_host->rec_y, hpu_, hp_pitch_, stream_);
    if (stream_m_) HIP_CHECK(hipEventRecord(ev_hpu_, stream_));
}

void GpuH264Encoder::enqueue_kernels(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish) {
    FrameSlot& sl = slots_[prep_slot_];
    enqueue_analysis_kernels(idr, src_y, src_uv, publish);
    async_frame_ = launcher_.joinable() && publish && !sync_launch_;
    if (async_frame_) {  // entropy chain to the launcher thread (its stream operations only there)
        HIP_CHECK(hipEventRecord(sl.analysis_done, stream_));
        hipEvent_t sse_ready = nullptr;
        if (sl.deblock) {
            unfiltered_planes(sl);
            launch_deblock(geom_, sl.buf, src_y, src_uv, stream_);
            HIP_CHECK(hipEventRecord(sl.deblock_done, stream_));
            sse_ready = sl.deblock_done;
        }
        if (stream_a_ && hpel_side_ && publish) {
            HIP_CHECK(hipEventRecord(ref_ready_, stream_));
            ref_seq_ = seq_;
        }
        HIP_CHECK(hipGetLastError());
        {
            std::lock_guard<std::mutex> lk(lmu_);
            if (lerr_) std::rethrow_exception(lerr_);
            ljobs_.push_back(EntropyJob{prep_slot_, sse_ready});
            slot_job_[prep_slot_] = ++l_pushed_;
        }
        lcv_.notify_all();
        return;
    }
    link_entropy();
    hipStream_t es = stream_e_ ? stream_e_ : stream_;
    hipEvent_t sse_ready = nullptr;
    if (sl.deblock) {  // in-loop filter on the analysis stream: the next frame predicts from it,
                         // while this frame's CAVLC runs beside it on the entropy stream
        unfiltered_planes(sl);
        launch_deblock(geom_, sl.buf, src_y, src_uv, stream_);
        if (stream_e_) {
            HIP_CHECK(hipEventRecord(sl.deblock_done, stream_));
            sse_ready = sl.deblock_done;
        }
    }
    if (stream_a_ && hpel_side_ && publish) {  // the next picture's reference is final
        HIP_CHECK(hipEventRecord(ref_ready_, stream_));
        ref_seq_ = seq_;
    }
    launch_entropy(geom_, sl.buf, sl.host_out, es, sse_ready);
    HIP_CHECK(hipGetLastError());
}

void GpuH264Encoder::fill_state(FrameSlot& sl, bool idr, int qp, int ref, int cur) {
    FrameState& f = *sl.fs_host;
    f.ref_y = rec_y_[ref];
    f.ref_uv = rec_uv_[ref];
    f.rec_y = rec_y_[cur];
    f.rec_uv = rec_uv_[cur];
    f.idr = idr ? 1 : 0;
    f.frame_num = common_.cur_frame_num();
    f.idr_pic_id = common_.cur_idr_pic_id();
    f.qp = qp;
    f.slice_rows = idr ? idr_slice_rows(geom_.mb_h) : geom_.mb_h;
    f.num_slices = (geom_.mb_h + f.slice_rows - 1) / f.slice_rows;
    f.search_range = me_range(cfg_.search_range);
    f.me_coarse = cfg_.me_coarse;
    f.intra4x4 = cfg_.intra4x4;
    f.subpel = cfg_.subpel;
    f.deblock_off = sl.deblock ? 0 : 1;
    if (++db_epoch_ == 0) db_epoch_ = 1;  // 32-bit tag (bits 32..63 of the hand-off words), never 0
    f.db_epoch = (int32_t)db_epoch_;
    f.pic_init_qp = common_.pic_init_qp();
    f.chroma_qp_offset = cfg_.chroma_qp_offset;
    f.log2_max_frame_num = common_.log2_max_frame_num();
    const size_t org = (size_t)kHpelPad * hp_pitch_ + kHpelPad;
    f.hp_pitch = hp_pitch_;
    f.aq = cfg_.aq;
    f.intra_in_p = cfg_.intra_in_p;
    f.partitions = cfg_.partitions ? 1 : 0;
    f.mask_mx0 = mask_mb_[0];
    f.mask_my0 = mask_mb_[1];
    f.mask_mx1 = mask_mb_[2];
    f.mask_my1 = mask_mb_[3];
    f.hp_f = hp_[0] + org;
    f.hp_h = hp_[1] + org;
    f.hp_v = hp_[2] + org;
    f.hp_j = hp_[3] + org;
    f.me_f = sl.me_unf ? hpu_[0] + org : nullptr;
    f.me_h = sl.me_unf ? hpu_[1] + org : nullptr;
    f.me_v = sl.me_unf ? hpu_[2] + org : nullptr;
    f.me_j = sl.me_unf ? hpu_[3] + org : nullptr;
    f.sse_part = sl.buf.sse_part;
    f.prev_src = src_keep_[ref];
    f.save_src = src_keep_[cur];
}

int GpuH264Encoder::probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp) {
    // synchronous IDR encode of the first picture at `qp` (rate-control probe); touches no
    // stream state: the real first frame overwrites the reconstruction
    if (!inflight_.empty()) throw std::logic_error("GpuH264Encoder: probe with frames in flight");
    prep_slot_ = 0;
    FrameSlot& sl = slots_[0];
    sl.deblock = cfg_.deblock == 1;
    sl.me_unf = false;
    fill_state(sl, true, qp, cur_ ^ 1, cur_);
    sl.fs_host->frame_num = 0;
    sl.fs_host->idr_pic_id = 0;
    sync_launch_ = true;
    enqueue_kernels(true, src_y, src_uv, true);
    sync_launch_ = false;
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (stream_e_) HIP_CHECK(hipStreamSynchronize(stream_e_));
    const OutHeader hdr = *reinterpret_cast<const OutHeader*>(sl.host_out);
    // + start code, NAL header and a rough emulation-prevention allowance per slice
    return hdr.overflow ? (int)sl.buf.out_bytes : (int)(hdr.total_bytes + hdr.num_slices * 6 + 32);
}

bool GpuH264Encoder::prepare(bool force_idr) {
    if ((int)inflight_.size() >= depth_)
        throw std::logic_error("GpuH264Encoder: collect() a frame first (pipeline full)");
    const int s = (depth_ == 1) ? 0 : next_slot_;
    next_slot_ = (next_slot_ + 1) % depth_;
    prep_slot_ = s;
    ++seq_;
    FrameSlot& sl = slots_[s];
    common_.begin_frame(force_idr || !have_ref_);
    have_ref_ = true;  // this frame becomes the reference of the next one
    const bool idr = common_.cur_idr();
    sl.idr = idr;
    sl.qp = common_.cur_qp();
    const int ref = cur_;
    cur_ ^= 1;
    sl.fidx = seq_;
    sl.me_unf = !idr && last_deblock_;
    sl.deblock = db_lag_.decide((long long)seq_, idr);
    last_deblock_ = sl.deblock;
    fill_state(sl, idr, sl.qp, ref, cur_);
    return idr;
}

void GpuH264Encoder::enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    // hipGraph form: frame-state upload node + kernels that read the device copy (depends
    // only on fixed buffers, so with depth 1 the same graph replays every frame of a type)
    drain_launcher();
    FrameSlot& sl = slots_[prep_slot_];
    HIP_CHECK(hipMemcpyAsync(sl.buf.fs, sl.fs_host, sizeof(FrameState), hipMemcpyHostToDevice, stream_));
    enqueue_kernels(idr, src_y, src_uv, false);
}

void GpuH264Encoder::enqueue_analysis(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    drain_launcher();
    FrameSlot& sl = slots_[prep_slot_];
    HIP_CHECK(hipMemcpyAsync(sl.buf.fs, sl.fs_host, sizeof(FrameState), hipMemcpyHostToDevice, stream_));
    enqueue_analysis_kernels(idr, src_y, src_uv, false);
}

// GPU time comes from the device clock stamps in OutHeader (t_start by the first kernel, t_end by
// k_pack): no event between the kernels of a frame
void GpuH264Encoder::record_start() {}

void GpuH264Encoder::record_done() {
    FrameSlot& sl = slots_[prep_slot_];
    if (async_frame_) {
        async_frame_ = false;  // the launcher records sl.done after the entropy kernels
    } else {
        slot_job_[prep_slot_] = 0;
        HIP_CHECK(hipEventRecord(sl.done, stream_e_ ? stream_e_ : stream_));
    }
    inflight_.push_back(prep_slot_);
}

void GpuH264Encoder::submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr) {
    while (common_.wants_probe()) {
        const int q = common_.probe_qp();
        common_.add_probe(q, probe_bytes(src_y, src_uv, q));
    }
    const bool idr = prepare(force_idr);
    record_start();
    enqueue_kernels(idr, src_y, src_uv, true);  // eager: the state travels as kernel arguments
    record_done();
}

const std::vector<uint8_t>& GpuH264Encoder::collect() {
    if (inflight_.empty()) throw std::logic_error("GpuH264Encoder: nothing submitted");
    const int s = inflight_.front();
    inflight_.pop_front();
    FrameSlot& sl = slots_[s];
    wait_launched(s);
    wait_event(sl.done);
    last_done_ = sl.done;
    const OutHeader hdr = *reinterpret_cast<const OutHeader*>(sl.host_out);
    last_t_end_ = hdr.t_end;
    const double ms = hdr.t_end > hdr.t_start ? (double)(hdr.t_end - hdr.t_start) / clock_khz_ : 0.0;
    if (*sl.buf.db_err) {  // a deblocking hand-off spin timed out: the reference is unreliable
        *sl.buf.db_err = 0;
        common_.end_frame(0, sl.idr);
        have_ref_ = false;
        throw std::runtime_error("h264 gpu encoder: deblocking hand-off timed out");
    }
    if (hdr.overflow) {
        common_.end_frame(0, sl.idr);
        have_ref_ = false;  // reference is incomplete: next frame must be IDR
        throw std::runtime_error("h264 gpu encoder: output overflow (flags " + std::to_string(hdr.overflow) + ")");
    }
    const uint32_t* soff = reinterpret_cast<const uint32_t*>(sl.host_out + sizeof(OutHeader));
    const uint32_t* slen = soff + kMaxSlices;
    const uint8_t* payload = sl.host_out + kOutPayloadOffset;
    au_.clear();
    au_.reserve(hdr.total_bytes + hdr.total_bytes / 64 + 256);
    if (sl.idr) common_.write_parameter_sets(au_);
    for (uint32_t k = 0; k < hdr.num_slices; ++k) common_.write_slice_nal(au_, payload + soff[k], slen[k], sl.idr);
    stats_.frame_index = common_.frames();
    stats_.idr = sl.idr;
    stats_.qp = sl.qp;
    stats_.bytes = (int)au_.size();
    stats_.encode_ms = ms;
    for (int c = 0; c < 3; ++c) stats_.sse[c] = hdr.sse[c];
    stats_.sse_masked = hdr.sse_masked;
    stats_.masked_pixels = masked_pixels_;
    stats_.deblocked = (int)hdr.deblocked;
    stats_.db_coherent = (int)hdr.db_coherent;
    stats_.db_changed = (int)hdr.db_changed;
    stats_.db_moving = (int)hdr.db_moving;
    // picture fidx + kDbLag's filter, from this one's classes
    db_lag_.record((long long)sl.fidx, sl.idr, DbAutoCounts{hdr.db_coherent, hdr.db_changed, hdr.db_moving},
                   geom_.mb_w * geom_.mb_h);
    common_.end_frame((int)au_.size(), sl.idr);
    return au_;
}

}  // namespace h264
}  // namespace mx
