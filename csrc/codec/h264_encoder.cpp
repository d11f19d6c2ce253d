// Host driver of the HIP H.264 encoder + the Annex-B / rate-control logic shared with
// the CPU encoder.  See h264_gpu.h for the kernel chain.
#include "h264_encoder.h"

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
    rc_qp_ = cur_qp_;
}

void EncoderCommon::begin_frame(bool force_idr) {
    const bool idr = idr_requested_ || force_idr || frame_index_ == 0 ||
                     (cfg_.keyint > 0 && since_idr_ >= cfg_.keyint);
    cur_idr_ = idr;
    idr_requested_ = false;
    if (idr) {
        frame_num_ = 0;
        idr_pic_id_ = (idr_pic_id_ + 1) & 0xffff;
        since_idr_ = 0;
    } else {
        frame_num_ = (frame_num_ + 1) % (1 << log2_max_frame_num());
    }
    int q = (int)std::lround(rc_qp_);
    if (cfg_.bitrate_kbps > 0) q = std::clamp(q, cfg_.qp_min, cfg_.qp_max);
    cur_qp_ = std::clamp(q, 0, 51);
}

void EncoderCommon::end_frame(int bytes) {
    ++frame_index_;
    ++since_idr_;
    if (cfg_.bitrate_kbps <= 0) return;
    const double target = cfg_.bitrate_kbps * 1000.0 / std::max(1, cfg_.fps);
    const double bits = bytes * 8.0;
    vbv_fill_ = std::max(0.0, vbv_fill_ + bits - target);
    // cap the virtual buffer at ~0.5 s so a burst cannot pin the QP forever
    vbv_fill_ = std::min(vbv_fill_, target * std::max(1, cfg_.fps) * 0.5);
    if (cur_idr_) return;  // I frames are expected to be large; steer on P frames
    const double ratio = (bits + 0.25 * vbv_fill_ + 1.0) / target;
    const double step = std::clamp(6.0 * std::log2(ratio) * 0.25, -1.0, 1.5);
    rc_qp_ = std::clamp(rc_qp_ + step, (double)cfg_.qp_min, (double)cfg_.qp_max);
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

void EncoderCommon::write_slice_nal(std::vector<uint8_t>& out, const uint8_t* rbsp, size_t n) const {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back(cur_idr_ ? 0x65 : 0x41);  // IDR slice (ref_idc 3) / non-IDR slice (ref_idc 2)
    emulation_prevent(out, rbsp, n);
}

// ------------------------------------------------------------------ GpuH264Encoder
GpuH264Encoder::GpuH264Encoder(const EncoderConfig& cfg, hipStream_t stream)
    : cfg_(cfg), common_(cfg), stream_(stream) {
    geom_.width = cfg.width;
    geom_.height = cfg.height;
    geom_.mb_w = common_.mb_w();
    geom_.mb_h = common_.mb_h();
    geom_.coded_w = geom_.mb_w * 16;
    geom_.coded_h = geom_.mb_h * 16;
    geom_.pitch = (geom_.coded_w + 255) & ~255;
    if (geom_.mb_h > kMaxSlices) throw std::invalid_argument("picture too tall");
    const int nmb = geom_.mb_w * geom_.mb_h;
    const size_t ysz = (size_t)geom_.pitch * geom_.coded_h, uvsz = ysz / 2;
    for (int i = 0; i < 2; ++i) {
        HIP_CHECK(hipMalloc(&rec_y_[i], ysz));
        HIP_CHECK(hipMalloc(&rec_uv_[i], uvsz));
        HIP_CHECK(hipMemsetAsync(rec_y_[i], 16, ysz, stream_));
        HIP_CHECK(hipMemsetAsync(rec_uv_[i], 128, uvsz, stream_));
    }
    hp_pitch_ = (geom_.coded_w + 2 * kHpelPad + 255) & ~255;
    const size_t hp_bytes = (size_t)hp_pitch_ * (geom_.coded_h + 2 * kHpelPad);
    for (int i = 0; i < 4; ++i) HIP_CHECK(hipMalloc(&hp_[i], hp_bytes));
    HIP_CHECK(hipMalloc(&buf_.fs, sizeof(FrameState)));
    HIP_CHECK(hipMalloc(&buf_.mb, sizeof(MbInfo) * nmb));
    HIP_CHECK(hipMemsetAsync(buf_.mb, 0, sizeof(MbInfo) * nmb, stream_));
    HIP_CHECK(hipMalloc(&buf_.coef, sizeof(int16_t) * kCoefStride * nmb));
    HIP_CHECK(hipMalloc(&buf_.slot, sizeof(uint32_t) * kSlotWords * (size_t)nmb));
    HIP_CHECK(hipMalloc(&buf_.slot_bits, sizeof(uint32_t) * nmb));
    HIP_CHECK(hipMalloc(&buf_.unit_off, sizeof(uint32_t) * nmb));
    HIP_CHECK(hipMalloc(&buf_.skip_run, sizeof(int32_t) * nmb));
    HIP_CHECK(hipMalloc(&buf_.coded_list, sizeof(uint32_t) * nmb));
    HIP_CHECK(hipMalloc(&buf_.coded_info, sizeof(uint4) * nmb));
    HIP_CHECK(hipMalloc(&buf_.slice_info, sizeof(uint32_t) * kSliceInfo * kMaxSlices));
    HIP_CHECK(hipMemsetAsync(buf_.slice_info, 0, sizeof(uint32_t) * kSliceInfo * kMaxSlices, stream_));
    // payload capacity: 768 B per MB (intra at low QP stays far below)
    buf_.out_bytes = (size_t)nmb * 768;
    HIP_CHECK(hipMalloc(&buf_.out_hdr, sizeof(OutHeader)));
    if ((nmb + 3) / 4 > kSsePartStride) throw std::invalid_argument("frame too large for the distortion partials");
    HIP_CHECK(hipMalloc(&buf_.sse_part, 3 * sizeof(unsigned long long) * kSsePartStride));
    HIP_CHECK(hipHostMalloc(&fs_host_, sizeof(FrameState), hipHostMallocDefault));
    host_out_bytes_ = kOutPayloadOffset + buf_.out_bytes + 16;
    HIP_CHECK(hipHostMalloc(&host_out_, host_out_bytes_, hipHostMallocMapped));
    std::memset(host_out_, 0, kOutPayloadOffset);
    HIP_CHECK(hipEventCreate(&done_));
    HIP_CHECK(hipEventCreate(&start_));
    HIP_CHECK(hipStreamSynchronize(stream_));
}

GpuH264Encoder::~GpuH264Encoder() {
    hipStreamSynchronize(stream_);
    for (int i = 0; i < 2; ++i) {
        hipFree(rec_y_[i]);
        hipFree(rec_uv_[i]);
    }
    for (int i = 0; i < 4; ++i) hipFree(hp_[i]);
    hipFree(buf_.fs);
    hipFree(buf_.mb);
    hipFree(buf_.coef);
    hipFree(buf_.slot);
    hipFree(buf_.slot_bits);
    hipFree(buf_.unit_off);
    hipFree(buf_.skip_run);
    hipFree(buf_.coded_list);
    hipFree(buf_.coded_info);
    hipFree(buf_.slice_info);
    hipFree(buf_.out_hdr);
    hipFree(buf_.sse_part);
    hipHostFree(fs_host_);
    hipHostFree(host_out_);
    hipEventDestroy(done_);
    hipEventDestroy(start_);
}

void GpuH264Encoder::enqueue_kernels(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    if (idr) {
        launch_intra(geom_, buf_, src_y, src_uv, stream_);
    } else {
        launch_hpel(geom_, buf_, hp_, hp_pitch_, stream_);
        launch_me(geom_, buf_, src_y, stream_);
        launch_inter(geom_, buf_, src_y, src_uv, stream_);
    }
    launch_entropy(geom_, buf_, host_out_, stream_);
    HIP_CHECK(hipGetLastError());
}

bool GpuH264Encoder::prepare(bool force_idr) {
    if (pending_) throw std::logic_error("GpuH264Encoder: collect() the previous frame first");
    common_.begin_frame(force_idr || !have_ref_);
    const bool idr = common_.cur_idr();
    const int ref = cur_;
    cur_ ^= 1;
    FrameState& f = *fs_host_;
    f.ref_y = rec_y_[ref];
    f.ref_uv = rec_uv_[ref];
    f.rec_y = rec_y_[cur_];
    f.rec_uv = rec_uv_[cur_];
    f.idr = idr ? 1 : 0;
    f.frame_num = common_.cur_frame_num();
    f.idr_pic_id = common_.cur_idr_pic_id();
    f.qp = common_.cur_qp();
    f.slice_rows = idr ? 1 : geom_.mb_h;
    f.num_slices = idr ? geom_.mb_h : 1;
    f.search_range = me_range(cfg_.search_range);
    f.subpel = cfg_.subpel;
    f.deblock_off = 1;
    f.pic_init_qp = common_.pic_init_qp();
    f.chroma_qp_offset = cfg_.chroma_qp_offset;
    f.log2_max_frame_num = common_.log2_max_frame_num();
    const size_t org = (size_t)kHpelPad * hp_pitch_ + kHpelPad;
    f.hp_pitch = hp_pitch_;
    f.hp_f = hp_[0] + org;
    f.hp_h = hp_[1] + org;
    f.hp_v = hp_[2] + org;
    f.hp_j = hp_[3] + org;
    f.sse_part = buf_.sse_part;
    return idr;
}

void GpuH264Encoder::enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    // everything here depends only on fixed buffers + the device frame state, so the same
    // sequence can be captured once into a hipGraph and replayed every frame
    HIP_CHECK(hipMemcpyAsync(buf_.fs, fs_host_, sizeof(FrameState), hipMemcpyHostToDevice, stream_));
    enqueue_kernels(idr, src_y, src_uv);
}

void GpuH264Encoder::record_start() { HIP_CHECK(hipEventRecord(start_, stream_)); }

void GpuH264Encoder::record_done() {
    HIP_CHECK(hipEventRecord(done_, stream_));
    pending_ = true;
}

void GpuH264Encoder::submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr) {
    const bool idr = prepare(force_idr);
    record_start();
    enqueue_body(idr, src_y, src_uv);
    record_done();
}

const std::vector<uint8_t>& GpuH264Encoder::collect() {
    if (!pending_) throw std::logic_error("GpuH264Encoder: nothing submitted");
    HIP_CHECK(hipEventSynchronize(done_));
    pending_ = false;
    float ms = 0;
    hipEventElapsedTime(&ms, start_, done_);
    const OutHeader hdr = *reinterpret_cast<const OutHeader*>(host_out_);
    if (hdr.overflow) {
        common_.end_frame(0);
        have_ref_ = false;  // reference is incomplete: next frame must be IDR
        throw std::runtime_error("h264 gpu encoder: output overflow (flags " + std::to_string(hdr.overflow) + ")");
    }
    const uint32_t* soff = reinterpret_cast<const uint32_t*>(host_out_ + sizeof(OutHeader));
    const uint32_t* slen = soff + kMaxSlices;
    const uint8_t* payload = host_out_ + kOutPayloadOffset;
    au_.clear();
    au_.reserve(hdr.total_bytes + hdr.total_bytes / 64 + 256);
    if (common_.cur_idr()) common_.write_parameter_sets(au_);
    for (uint32_t s = 0; s < hdr.num_slices; ++s) common_.write_slice_nal(au_, payload + soff[s], slen[s]);
    stats_.frame_index = common_.frames();
    stats_.idr = common_.cur_idr();
    stats_.qp = common_.cur_qp();
    stats_.bytes = (int)au_.size();
    stats_.encode_ms = ms;
    for (int c = 0; c < 3; ++c) stats_.sse[c] = hdr.sse[c];
    common_.end_frame((int)au_.size());
    have_ref_ = true;
    return au_;
}

}  // namespace h264
}  // namespace mx
