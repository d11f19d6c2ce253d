// Host driver of the HIP HEVC encoder (kernel chain in hevc_kernels.hip).  Mirrors the
// H.264 driver: per-frame slots (pinned frame state, zero-copy output), optional second
// HIP stream for entropy coding so frame n's CABAC overlaps frame n+1's analysis.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../common/hip_check.h"
#include "h264_mb.h"
#include "hevc_encoder.h"

namespace mx {
namespace hevc {

void GpuHevcEncoder::alloc_slot(FrameSlot& sl) {
    const int ncu = geom_.mb_w * geom_.mb_h;                // 16x16 units
    const int nctb = common_.num_ctbs(), npos = 4 * nctb;  // 32x32 CTBs, coding positions
    // substreams: cost-balanced slices, or (WPP) every CTB row
    const int ns = cfg_.hevc_wpp ? std::max(common_.max_slices(), common_.c32_h()) : common_.max_slices();
    HevcDeviceBuffers& b = sl.buf;
    HIP_CHECK(hipMalloc(&b.fs, sizeof(HevcFrameState)));
    HIP_CHECK(hipMalloc(&b.me.fs, sizeof(h264::FrameState)));
    HIP_CHECK(hipMalloc(&b.me.mb, sizeof(h264::MbInfo) * ncu));
    HIP_CHECK(hipMemsetAsync(b.me.mb, 0, sizeof(h264::MbInfo) * ncu, stream_));
    HIP_CHECK(hipMalloc(&b.cu, sizeof(CuInfo) * ncu));
    HIP_CHECK(hipMalloc(&b.coef, sizeof(int16_t) * kCoefPerCu * (size_t)ncu));
    // per-substream CABAC output slot: room for 1 KiB per unit of an even share of the picture plus
    // one slice of CTB rows (slices are cost-balanced, so a slice of many cheap CTBs stays small)
    const size_t units_per_slot = std::max((size_t)(ncu + ns - 1) / ns + (size_t)2 * common_.slice_rows() * geom_.mb_w,
                                           (size_t)2 * geom_.mb_w);
    b.slice_cap = (uint32_t)((units_per_slot * 1024 + 15) & ~(size_t)15);
    HIP_CHECK(hipMalloc(&b.slice_data, (size_t)b.slice_cap * ns));
    HIP_CHECK(hipMalloc(&b.slice_len, sizeof(uint32_t) * ns));
    HIP_CHECK(hipMalloc(&b.slice_first, sizeof(int) * ns));
    HIP_CHECK(hipMalloc(&b.slice_of_cu, sizeof(int) * nctb));
    HIP_CHECK(hipMalloc(&b.nslices, sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&b.qpy, ncu));
    HIP_CHECK(hipMalloc(&b.qp_pred, ncu));
    HIP_CHECK(hipMalloc(&b.imode, ncu));
    // arrays scanned in 4096-entry tiles of 16-byte loads (per CTB costs, per coding position token
    // counts): padded with zeros to a whole tile
    auto pad = [](size_t n) { return (n + kScanTilePad - 1) / kScanTilePad * kScanTilePad + 4; };
    const size_t nctb_pad = pad((size_t)nctb), npos_pad = pad((size_t)npos);
    HIP_CHECK(hipMalloc(&b.cost, sizeof(uint32_t) * nctb_pad));
    HIP_CHECK(hipMemsetAsync(b.cost, 0, sizeof(uint32_t) * nctb_pad, stream_));
    HIP_CHECK(hipMalloc(&b.qpc, ncu));
    HIP_CHECK(hipMalloc(&b.sao, sizeof(uint32_t) * 4 * (size_t)nctb));
    HIP_CHECK(hipMalloc(&b.slice_clk, sizeof(unsigned long long) * 2 * (size_t)ns));
    HIP_CHECK(hipMalloc(&b.tok, sizeof(uint16_t) * kMaxCuTokens * (size_t)npos));
    HIP_CHECK(hipMalloc(&b.ntok, sizeof(uint32_t) * npos_pad));
    HIP_CHECK(hipMemsetAsync(b.ntok, 0, sizeof(uint32_t) * npos_pad, stream_));
    HIP_CHECK(hipMalloc(&b.tok_off, sizeof(uint32_t) * npos_pad));
    // + one chunk of padding: k_hevc_arith reads whole 256-token chunks
    HIP_CHECK(hipMalloc(&b.tok_dense, sizeof(uint16_t) * (kMaxCuTokens * (size_t)npos + 512)));
    HIP_CHECK(hipMalloc(&b.sse_part, 4 * sizeof(unsigned long long) * h264::kSsePartStride));
    HIP_CHECK(hipMalloc(&b.sse_tot, kSseSlots * kSseSlotWords * sizeof(unsigned long long)));
    HIP_CHECK(hipMalloc(&b.pack_done, sizeof(uint32_t)));
    HIP_CHECK(hipMemsetAsync(b.pack_done, 0, sizeof(uint32_t), stream_));
    HIP_CHECK(hipMalloc(&b.wpp_ctx, sizeof(uint32_t) * kWppCtxWords * (size_t)common_.c32_h()));
    HIP_CHECK(hipMalloc(&b.wpp_flag, sizeof(uint32_t) * (size_t)common_.c32_h()));
    HIP_CHECK(hipMemsetAsync(b.wpp_flag, 0, sizeof(uint32_t) * (size_t)common_.c32_h(), stream_));
    b.db_state = db_state_;
    HIP_CHECK(hipHostMalloc(&b.wpp_err, sizeof(int), hipHostMallocMapped));
    *b.wpp_err = 0;
    b.out_bytes = (size_t)ncu * 768;
    HIP_CHECK(hipHostMalloc(&sl.fs_host, sizeof(HevcFrameState), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc(&sl.me_fs_host, sizeof(h264::FrameState), hipHostMallocDefault));
    std::memset(sl.me_fs_host, 0, sizeof(h264::FrameState));
    HIP_CHECK(hipHostMalloc(&sl.host_out, kOutPayloadOffset + b.out_bytes + 16, hipHostMallocMapped));
    std::memset(sl.host_out, 0, kOutPayloadOffset);
    HIP_CHECK(hipEventCreate(&sl.start));
    HIP_CHECK(hipEventCreateWithFlags(&sl.analysis_done, hipEventDisableTiming));
    HIP_CHECK(hipEventCreate(&sl.done));
}

void GpuHevcEncoder::free_slot(FrameSlot& sl) {
    HevcDeviceBuffers& b = sl.buf;
    for (void* p : {(void*)b.fs, (void*)b.me.fs, (void*)b.me.mb, (void*)b.cu, (void*)b.coef, (void*)b.slice_data,
                    (void*)b.slice_len, (void*)b.slice_first, (void*)b.slice_of_cu, (void*)b.nslices, (void*)b.qpy, (void*)b.qp_pred, (void*)b.imode, (void*)b.cost, (void*)b.qpc,
                    (void*)b.sse_part, (void*)b.sse_tot, (void*)b.sao, (void*)b.slice_clk, (void*)b.tok, (void*)b.ntok, (void*)b.tok_off,
                    (void*)b.tok_dense, (void*)b.wpp_ctx, (void*)b.wpp_flag, (void*)b.pack_done})
        if (p) (void)hipFree(p);
    if (b.wpp_err) (void)hipHostFree(b.wpp_err);
    if (sl.fs_host) (void)hipHostFree(sl.fs_host);
    if (sl.me_fs_host) (void)hipHostFree(sl.me_fs_host);
    if (sl.host_out) (void)hipHostFree(sl.host_out);
    for (hipEvent_t e : {sl.start, sl.analysis_done, sl.done})
        if (e) (void)hipEventDestroy(e);
}

GpuHevcEncoder::GpuHevcEncoder(const EncoderConfig& cfg, hipStream_t stream)
    : cfg_(cfg.with_aq_default(6)), common_(cfg), stream_(stream) {
    if (cfg.pipeline_depth < 1 || cfg.pipeline_depth > kMaxInFlight)
        throw std::invalid_argument("pipeline_depth must be 1, 2 or 3");
    if (2 * common_.slice_rows() > kMaxSliceRows) throw std::invalid_argument("hevc: too many CTB rows per slice");
    depth_ = cfg.pipeline_depth;
    geom_.width = cfg.width;
    geom_.height = cfg.height;
    geom_.mb_w = common_.ctb_w();
    geom_.mb_h = common_.ctb_h();
    geom_.coded_w = geom_.mb_w * kCtb;
    geom_.coded_h = geom_.mb_h * kCtb;
    geom_.pitch = (geom_.coded_w + 255) & ~255;
    const int ncu = geom_.mb_w * geom_.mb_h;
    if (std::max((ncu + 3) / 4, common_.num_ctbs()) > h264::kSsePartStride)
        throw std::invalid_argument("frame too large for the distortion partials");
    bl_safe_ = bl_safe_modes(4, 0) & bl_safe_modes(3, 1);
    bl_safe_split_ = bl_safe_split();
    const size_t ysz = (size_t)geom_.pitch * geom_.coded_h, uvsz = ysz / 2;
    for (int i = 0; i < 2; ++i) {
        HIP_CHECK(hipMalloc(&rec_y_[i], ysz));
        HIP_CHECK(hipMalloc(&rec_uv_[i], uvsz));
        HIP_CHECK(hipMemsetAsync(rec_y_[i], 16, ysz, stream_));
        HIP_CHECK(hipMemsetAsync(rec_uv_[i], 128, uvsz, stream_));
        HIP_CHECK(hipMalloc(&src_keep_[i], ysz));
        HIP_CHECK(hipMemsetAsync(src_keep_[i], 16, ysz, stream_));
    }
    if (cfg.sao) {
        HIP_CHECK(hipMalloc(&pre_y_, ysz));
        HIP_CHECK(hipMalloc(&pre_uv_, uvsz));
    }
    if (cfg.mask_x1 > cfg.mask_x0 && cfg.mask_y1 > cfg.mask_y0) {  // CTB = 16: the H.264 MB-aligned region
        mask_c_[0] = std::max(0, cfg.mask_x0) / kCtb;
        mask_c_[1] = std::max(0, cfg.mask_y0) / kCtb;
        mask_c_[2] = std::min(geom_.mb_w, (cfg.mask_x1 + kCtb - 1) / kCtb);
        mask_c_[3] = std::min(geom_.mb_h, (cfg.mask_y1 + kCtb - 1) / kCtb);
    }
    masked_pixels_ = (int64_t)cfg.width * cfg.height;
    for (int cy = mask_c_[1]; cy < mask_c_[3]; ++cy)
        for (int cx = mask_c_[0]; cx < mask_c_[2]; ++cx)
            masked_pixels_ -= (int64_t)std::max(0, std::min(kCtb, cfg.width - kCtb * cx)) *
                              std::max(0, std::min(kCtb, cfg.height - kCtb * cy));
    hp_pitch_ = (geom_.coded_w + 2 * h264::kHpelPad + 255) & ~255;
    const size_t hp_bytes = (size_t)hp_pitch_ * (geom_.coded_h + 2 * h264::kHpelPad);
    for (int i = 0; i < 4; ++i) HIP_CHECK(hipMalloc(&hp_[i], hp_bytes));
    HIP_CHECK(hipMalloc(&db_state_, sizeof(uint32_t) * 4));
    HIP_CHECK(hipMemsetAsync(db_state_, 0, sizeof(uint32_t) * 4, stream_));
    for (int i = 0; i < depth_; ++i) alloc_slot(slots_[i]);
    if (depth_ > 1) {
        // entropy streams: MXDESK_HEVC_ESTREAMS of them, slots beyond share them round-robin.  Every
        // stream of a process takes a hardware queue (GPU_MAX_HW_QUEUES, 4 by default) and streams
        // beyond that share queues in turn, so the default leaves two queues to the analysis and the
        // capture stream: a capture stream sharing the analysis queue serialises the render with the
        // analysis (4K depth 3: 1,657 fps with three entropy streams, 2,277 with two; no capture
        // stream and three: 2,176 -- profiles/r06_streams)
        const char* ne = std::getenv("MXDESK_HEVC_ESTREAMS");
        const char* hq = std::getenv("GPU_MAX_HW_QUEUES");
        const int queues = hq && std::atoi(hq) > 0 ? std::atoi(hq) : 4;
        n_es_ = std::clamp(ne ? std::atoi(ne) : std::min(depth_, queues - 2), 1, depth_);
        for (int i = 0; i < n_es_; ++i) HIP_CHECK(hipStreamCreateWithFlags(&stream_e_[i], hipStreamNonBlocking));
        for (int i = n_es_; i < depth_; ++i) stream_e_[i] = stream_e_[i % n_es_];
    }
    clock_khz_ = device_clock_khz();
    HIP_CHECK(hipStreamSynchronize(stream_));
}

GpuHevcEncoder::~GpuHevcEncoder() {
    (void)hipStreamSynchronize(stream_);
    for (int i = 0; i < n_es_; ++i) {
        (void)hipStreamSynchronize(stream_e_[i]);
        (void)hipStreamDestroy(stream_e_[i]);
    }
    for (int i = 0; i < 2; ++i) {
        (void)hipFree(rec_y_[i]);
        (void)hipFree(rec_uv_[i]);
        (void)hipFree(src_keep_[i]);
    }
    for (int i = 0; i < 4; ++i) (void)hipFree(hp_[i]);
    if (pre_y_) (void)hipFree(pre_y_);
    if (pre_uv_) (void)hipFree(pre_uv_);
    for (int i = 0; i < depth_; ++i) free_slot(slots_[i]);
    if (db_state_) (void)hipFree(db_state_);
}

void GpuHevcEncoder::fill_state(FrameSlot& sl, bool idr, int qp, int ref, int cur, bool probe) {
    const size_t org = (size_t)h264::kHpelPad * hp_pitch_ + h264::kHpelPad;
    HevcFrameState& f = *sl.fs_host;
    f.ref_y = rec_y_[ref];
    f.ref_uv = rec_uv_[ref];
    // the rate-control probe codes without SAO (as the CPU encoder's probe)
    f.sao = (cfg_.sao && !probe) ? 1 : 0;
    f.deblock_on = cfg_.hevc_deblock() ? 1 : 0;  // adaptive: k_hevc_db_auto overwrites it on the device
    f.deblock_auto = cfg_.hevc_deblock_auto() ? 1 : 0;
    f.chroma_keep = cfg_.hevc_chroma_keep ? 1 : 0;
    f.rec_y = f.sao ? pre_y_ : rec_y_[cur];
    f.rec_uv = f.sao ? pre_uv_ : rec_uv_[cur];
    f.sao_y = rec_y_[cur];
    f.sao_uv = rec_uv_[cur];
    f.hp_f = hp_[0] + org;
    f.hp_pitch = hp_pitch_;
    f.idr = idr ? 1 : 0;
    f.qp = qp;
    f.slice_rows = 2 * common_.slice_rows();  // in 16x16-unit rows
    f.i_seg_w = common_.i_seg_w();
    f.num_slices = common_.num_slices();
    f.bl_safe = bl_safe_;
    f.bl_safe_split = bl_safe_split_;
    f.depth_inter = common_.depth_inter();
    f.depth_intra = common_.depth_intra();
    f.aq = cfg_.aq;
    f.tu_split = cfg_.tu_split;  // 0 none, 1 8x8 nodes, 2 also 4x4 luma TUs
    f.chroma_qp_offset = cfg_.chroma_qp_offset;
    // distortion partials: k_hevc_sao (totals) with SAO, else k_hevc_sse (one per unit row) after
    // deblocking, else the analysis kernels' (P: one per CTB, I: one per unit row)
    f.n_sse_parts = f.sao ? common_.num_ctbs()
                          : (cfg_.hevc_deblock() ? geom_.mb_h : (idr ? geom_.mb_h * common_.i_split() : common_.num_ctbs()));
    f.sse_part = sl.buf.sse_part;
    f.sse_tot = sl.buf.sse_tot;
    for (int k = 0; k < 4; ++k) f.mask_c[k] = mask_c_[k];
    f.prev_src = src_keep_[ref];
    f.save_src = src_keep_[cur];
    f.wpp = cfg_.hevc_wpp ? 1 : 0;
    f.wpp_rows = common_.wpp_rows();
    if (++wpp_epoch_ == 0) wpp_epoch_ = 1;
    f.wpp_epoch = wpp_epoch_;
    f.wpp_ctx = sl.buf.wpp_ctx;
    f.wpp_flag = sl.buf.wpp_flag;
    f.wpp_err = sl.buf.wpp_err;
    h264::FrameState& m = *sl.me_fs_host;  // motion search state (shared H.264 kernels)
    m.ref_y = rec_y_[ref];
    m.ref_uv = rec_uv_[ref];
    m.qp = qp;
    m.search_range = h264::me_range(cfg_.search_range);
    m.me_coarse = cfg_.me_coarse;
    m.subpel = cfg_.subpel;
    m.partitions = 0;  // HEVC codes 16x16 prediction units from the 16x16 vectors
    m.hp_pitch = hp_pitch_;
    m.hp_f = hp_[0] + org;
    m.hp_h = hp_[1] + org;
    m.hp_v = hp_[2] + org;
    m.hp_j = hp_[3] + org;
    m.sse_part = sl.buf.sse_part;
}

int GpuHevcEncoder::probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp) {
    // synchronous IDR encode of the first picture at `qp` (rate-control probe, see
    // h264::EncoderCommon); the real first frame overwrites the reconstruction
    if (!inflight_.empty()) throw std::logic_error("GpuHevcEncoder: probe with frames in flight");
    prep_slot_ = 0;
    FrameSlot& sl = slots_[0];
    fill_state(sl, true, qp, cur_ ^ 1, cur_, true);
    enqueue_body(true, src_y, src_uv);
    HIP_CHECK(hipStreamSynchronize(stream_));
    HIP_CHECK(hipStreamSynchronize(es(0)));
    const HevcOutHeader hdr = *reinterpret_cast<const HevcOutHeader*>(sl.host_out);
    if (hdr.overflow) return (int)sl.buf.out_bytes;
    // the exact substream lengths (total_bytes counts the 16-byte aligned payload slots), plus the
    // per-NAL allowance per slice, as the CPU encoder's probe: the two must pick the same QP
    const uint32_t* len = reinterpret_cast<const uint32_t*>(sl.host_out + sizeof(HevcOutHeader)) + kMaxSlices;
    size_t total = 0;
    for (uint32_t k = 0; k < hdr.num_slices && k < (uint32_t)kMaxSlices; ++k) total += len[k];
    return (int)(total + common_.num_slices() * 12 + 64);
}

bool GpuHevcEncoder::prepare(bool force_idr) {
    if ((int)inflight_.size() >= depth_) throw std::logic_error("GpuHevcEncoder: collect() a frame first (pipeline full)");
    const int s = (depth_ == 1) ? 0 : next_slot_;
    next_slot_ = (next_slot_ + 1) % depth_;
    prep_slot_ = s;
    FrameSlot& sl = slots_[s];
    h264::EncoderCommon& rc = common_.rc();
    rc.begin_frame(force_idr || !have_ref_);
    have_ref_ = true;
    const bool idr = rc.cur_idr();
    sl.idr = idr;
    sl.qp = rc.cur_qp();
    sl.poc = idr ? 0 : common_.poc();
    const int ref = cur_;
    cur_ ^= 1;
    fill_state(sl, idr, sl.qp, ref, cur_);
    return idr;
}

void GpuHevcEncoder::enqueue_analysis(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    enqueue_analysis_impl(idr, src_y, src_uv, false);
}

void GpuHevcEncoder::enqueue_analysis_impl(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish) {
    FrameSlot& sl = slots_[prep_slot_];
    HevcOutHeader* hdr = reinterpret_cast<HevcOutHeader*>(sl.host_out);
    if (publish) {  // eager: states as kernel arguments, start clock stamped on the device
        launch_hevc_publish(sl.buf, *sl.fs_host, idr ? nullptr : sl.me_fs_host, &hdr->t_start, stream_);
    } else {  // graph form: copy nodes from the pinned states (no start stamp)
        hdr->t_start = 0;
        HIP_CHECK(hipMemcpyAsync(sl.buf.fs, sl.fs_host, sizeof(HevcFrameState), hipMemcpyHostToDevice, stream_));
        if (!idr)
            HIP_CHECK(hipMemcpyAsync(sl.buf.me.fs, sl.me_fs_host, sizeof(h264::FrameState), hipMemcpyHostToDevice,
                                     stream_));
    }
    if (idr) {
        if (cfg_.aq >= 3)  // the next P picture's temporal classes compare against this source
            launch_hevc_save_src(geom_, sl.buf, src_y, stream_);
        launch_hevc_intra(geom_, sl.buf, 2 * common_.slice_rows(), common_.num_slices(), src_y, src_uv, stream_);
    } else {
        h264::launch_hpel(geom_, sl.buf.me, hp_, hp_pitch_, stream_);
        h264::launch_me(geom_, sl.buf.me, src_y, stream_);
        launch_hevc_inter(geom_, sl.buf, src_y, src_uv, stream_);
    }
    launch_hevc_layout(geom_, sl.buf, idr, common_.max_slices(), cfg_.hevc_slice_cost, cfg_.hevc_deblock(), sl.fs_host->sao != 0, src_y,
                       src_uv, stream_, cfg_.hevc_deblock_auto());
}

void GpuHevcEncoder::link_entropy() {
    if (!stream_e_[prep_slot_]) return;
    FrameSlot& sl = slots_[prep_slot_];
    HIP_CHECK(hipEventRecord(sl.analysis_done, stream_));
    HIP_CHECK(hipStreamWaitEvent(stream_e_[prep_slot_], sl.analysis_done, 0));
}

void GpuHevcEncoder::enqueue_entropy() {
    FrameSlot& sl = slots_[prep_slot_];
    launch_hevc_entropy(geom_, sl.buf, common_.max_slices(), sl.host_out, es(prep_slot_));
}

void GpuHevcEncoder::enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) {
    enqueue_analysis(idr, src_y, src_uv);
    link_entropy();
    enqueue_entropy();
    HIP_CHECK(hipGetLastError());
}

// eager frames time themselves with device clock stamps (k_hevc_publish / k_hevc_pack); graph
// frames keep the timing event
void GpuHevcEncoder::record_start() {
    if (!eager_) HIP_CHECK(hipEventRecord(slots_[prep_slot_].start, stream_));
}

void GpuHevcEncoder::record_done() {
    FrameSlot& sl = slots_[prep_slot_];
    HIP_CHECK(hipEventRecord(sl.done, es(prep_slot_)));
    inflight_.push_back(prep_slot_);
}

void GpuHevcEncoder::submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr) {
    h264::EncoderCommon& rc = common_.rc();
    while (rc.wants_probe()) {
        const int q = rc.probe_qp();
        rc.add_probe(q, probe_bytes(src_y, src_uv, q));
    }
    const bool idr = prepare(force_idr);
    eager_ = true;
    record_start();
    enqueue_analysis_impl(idr, src_y, src_uv, true);
    link_entropy();
    enqueue_entropy();
    HIP_CHECK(hipGetLastError());
    record_done();
    eager_ = false;
}

const std::vector<uint8_t>& GpuHevcEncoder::collect() {
    if (inflight_.empty()) throw std::logic_error("GpuHevcEncoder: nothing submitted");
    const int s = inflight_.front();
    inflight_.pop_front();
    FrameSlot& sl = slots_[s];
    wait_event(sl.done);
    last_done_ = sl.done;
    const HevcOutHeader hdr = *reinterpret_cast<const HevcOutHeader*>(sl.host_out);
    last_t_end_ = hdr.t_end;
    float ms = 0;
    if (hdr.t_start != 0)  // eager frame: device clock stamps
        ms = hdr.t_end > hdr.t_start ? (float)((double)(hdr.t_end - hdr.t_start) / clock_khz_) : 0.f;
    else
        (void)hipEventElapsedTime(&ms, sl.start, sl.done);
    h264::EncoderCommon& rc = common_.rc();
    if (hdr.overflow) {
        rc.end_frame(0, sl.idr);
        have_ref_ = false;  // reference incomplete: the next frame must be IDR
        throw std::runtime_error("hevc gpu encoder: output overflow");
    }
    if (*sl.buf.wpp_err) {  // a WPP substream gave up waiting for the row above: contexts unreliable
        *sl.buf.wpp_err = 0;
        rc.end_frame(0, sl.idr);
        have_ref_ = false;
        throw std::runtime_error("hevc gpu encoder: WPP context hand-off timed out");
    }
    // substream records: a slice each, or with WPP one per CTU row, grouped into slices by the
    // slice-start flag
    const uint32_t* soff = reinterpret_cast<const uint32_t*>(sl.host_out + sizeof(HevcOutHeader));
    const uint32_t* slen = soff + kMaxSlices;
    const uint32_t* saddr = soff + 2 * kMaxSlices;
    const uint8_t* payload = sl.host_out + kOutPayloadOffset;
    const uint32_t nsub = hdr.num_slices;
    last_slot_ = s;
    last_first_.resize(nsub);
    for (uint32_t k = 0; k < nsub; ++k) last_first_[k] = saddr[k] & ~kSubSliceStart;
    last_len_.assign(slen, slen + nsub);
    au_.clear();
    au_.reserve(hdr.total_bytes + hdr.total_bytes / 64 + 64 * nsub + 256);
    if (sl.idr) common_.write_parameter_sets(au_);
    if (!common_.wpp()) {
        for (uint32_t k = 0; k < nsub; ++k)
            common_.write_slice_nal(au_, (int)last_first_[k], sl.idr, sl.poc, sl.qp, hdr.deblocked != 0, payload + soff[k],
                                    slen[k]);
    } else {
        for (uint32_t k = 0; k < nsub;) {
            uint32_t e = k + 1, n = slen[k];
            while (e < nsub && !(saddr[e] & kSubSliceStart)) n += slen[e++];
            common_.write_slice_nal(au_, (int)last_first_[k], sl.idr, sl.poc, sl.qp, hdr.deblocked != 0, payload, n,
                                    slen + k, (int)(e - k), soff + k);
            k = e;
        }
    }
    stats_.frame_index = rc.frames();
    stats_.idr = sl.idr;
    stats_.qp = sl.qp;
    stats_.bytes = (int)au_.size();
    stats_.encode_ms = ms;
    for (int c = 0; c < 3; ++c) stats_.sse[c] = hdr.sse[c];
    stats_.sse_masked = hdr.sse_masked;
    stats_.masked_pixels = masked_pixels_;
    stats_.deblocked = (int)hdr.deblocked;
    rc.end_frame((int)au_.size(), sl.idr);
    return au_;
}

std::vector<std::array<uint64_t, 6>> GpuHevcEncoder::slice_timing() const {
    std::vector<std::array<uint64_t, 6>> out;
    if (last_slot_ < 0) return out;
    const size_t n = last_first_.size();
    const uint64_t nctb = (uint64_t)common_.num_ctbs();
    std::vector<unsigned long long> clk(2 * n);
    std::vector<uint32_t> off(4 * nctb + 1);
    HIP_CHECK(hipMemcpy(clk.data(), slots_[last_slot_].buf.slice_clk, sizeof(unsigned long long) * 2 * n,
                        hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(off.data(), slots_[last_slot_].buf.tok_off, sizeof(uint32_t) * (4 * nctb + 1),
                        hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (size_t k = 0; k < n; ++k) t0 = std::min(t0, clk[2 * k]);
    for (size_t k = 0; k < n; ++k) {  // (first CTB, CTBs, ...)
        const uint64_t end = k + 1 < n ? last_first_[k + 1] : nctb;
        out.push_back({last_first_[k], end - last_first_[k], last_len_[k], clk[2 * k + 1] - clk[2 * k],
                       clk[2 * k] - t0, off[4 * end] - off[4 * last_first_[k]]});
    }
    return out;
}

std::vector<std::array<uint32_t, 6>> GpuHevcEncoder::cu_token_table() const {
    std::vector<std::array<uint32_t, 6>> out;
    if (last_slot_ < 0) return out;
    const size_t ncu = (size_t)geom_.mb_w * geom_.mb_h, npos = 4 * (size_t)common_.num_ctbs();
    std::vector<CuInfo> cus(ncu);
    std::vector<uint32_t> ntok(npos);
    HIP_CHECK(hipMemcpy(cus.data(), slots_[last_slot_].buf.cu, sizeof(CuInfo) * ncu, hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(ntok.data(), slots_[last_slot_].buf.ntok, sizeof(uint32_t) * npos, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ncu; ++i) {
        const int kpos = cpos_of((int)(i % geom_.mb_w), (int)(i / geom_.mb_w), common_.c32_w());
        const CuInfo& c = cus[i];
        uint32_t lsum = 0, sb = 0;
        if (c.cbf & 1) lsum += c.last[0] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_y);
        if (c.cbf & 2) lsum += c.last[1] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_c[0]);
        if (c.cbf & 4) lsum += c.last[2] + 1u, sb += (uint32_t)__builtin_popcount(c.csbf_c[1]);
        out.push_back({c.type, c.cbf, lsum, sb, c.est_bytes, ntok[(size_t)kpos]});
    }
    return out;
}

}  // namespace hevc
}  // namespace mx
