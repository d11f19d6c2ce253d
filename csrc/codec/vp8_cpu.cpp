// CPU VP8 encoder: the decisions and arithmetic of the HIP kernels (vp8_kernels.hip), serially.
// The bit-exact oracle for the GPU encoder and the no-GPU fallback behind WEBRTC_ENCODER=vp8enc
// (the reference's libvpx `vp8enc`, README.md:21,35).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "h264_core.h"
#include "h264_mb.h"
#include "vp8_encoder.h"

namespace mx {
namespace vp8 {

namespace {

// Neighbour edges of the n x n block at (x0, y0) of a plane (cw x ch, interleave `step`, component
// offset `comp`) from the reconstruction, with VP8's frame-edge values.
Edge edge_of(const uint8_t* p, int pitch, int step, int comp, int x0, int y0, int n) {
    Edge e;
    e.have_above = y0 > 0;
    e.have_left = x0 > 0;
    for (int i = 0; i < n; ++i) {
        e.above[i] = y0 > 0 ? p[(y0 - 1) * pitch + (x0 + i) * step + comp] : 127;
        e.left[i] = x0 > 0 ? p[(y0 + i) * pitch + (x0 - 1) * step + comp] : 129;
    }
    e.corner = y0 == 0 ? 127 : (x0 == 0 ? 129 : p[(y0 - 1) * pitch + (x0 - 1) * step + comp]);
    return e;
}

}  // namespace

int lf_num_from_env() {
    const char* e = std::getenv("MXDESK_VP8_LF_NUM");
    return e && *e ? std::clamp(std::atoi(e), 0, 64) : kLfNumDefault;
}

CpuVp8Encoder::CpuVp8Encoder(const h264::EncoderConfig& cfg)
    : cfg_(cfg.with_aq_default(4)), common_(cfg), lf_(cfg.vp8_deblock_mode()), lf_num_(lf_num_from_env()) {
    mb_w_ = common_.mb_w();
    mb_h_ = common_.mb_h();
    cw_ = mb_w_ * 16;
    ch_ = mb_h_ * 16;
    for (int i = 0; i < 2; ++i) {
        rec_y_[i].assign((size_t)cw_ * ch_, 0);
        rec_uv_[i].assign((size_t)cw_ * ch_ / 2, 128);
    }
    mb_.resize((size_t)mb_w_ * mb_h_);
    lv_.resize(mb_.size() * kCoefPerMb);
}

void CpuVp8Encoder::analyse(const uint8_t* sy, const uint8_t* suv, int pitch, bool key, int qindex, int qp) {
    const Quant Q = quant_of(qindex);
    if (cfg_.aq >= 3) next_src_.assign((size_t)cw_ * ch_, 0);
    uint8_t* ry = rec_y_[cur_].data();
    uint8_t* ruv = rec_uv_[cur_].data();
    const uint8_t* fy = rec_y_[cur_ ^ 1].data();
    const uint8_t* fuv = rec_uv_[cur_ ^ 1].data();
    for (int mby = 0; mby < mb_h_; ++mby)
        for (int mbx = 0; mbx < mb_w_; ++mbx) {
            const int i = mby * mb_w_ + mbx, x0 = mbx * 16, y0 = mby * 16;
            Vp8Mb& m = mb_[i];
            std::memset(&m, 0, sizeof m);
            int16_t* lv = lv_.data() + (size_t)i * kCoefPerMb;
            int pred[256], res[256], rec[256], cp[2][64], cres[2][64], crec[2][64];
            uint32_t bpred_nz = 0;  // B_PRED: the luma blocks' non-zero bits (luma coded already, no Y2)
            if (key) {
                const Edge e = edge_of(ry, cw_, 1, 0, x0, y0, 16);
                const int dc = dc_of(e, 16);
                uint32_t best = ~0u;
                for (int mode = 0; mode < 4; ++mode) {
                    uint32_t sad = 0;
                    for (int y = 0; y < 16; ++y)
                        for (int x = 0; x < 16; ++x)
                            sad += (uint32_t)std::abs((int)sy[(y0 + y) * pitch + x0 + x] - pred_px(mode, e, 16, x, y, dc));
                    if (sad < best) {
                        best = sad;
                        m.ymode = (uint8_t)mode;
                    }
                }
                for (int y = 0; y < 16; ++y)
                    for (int x = 0; x < 16; ++x) pred[y * 16 + x] = pred_px(m.ymode, e, 16, x, y, dc);
                uint32_t lo = 0, hi = 0;  // B_PRED: the open-loop plan, then the closed-loop coding
                auto src = [&](int x, int y) { return (int)sy[(size_t)y * pitch + x]; };
                if (cfg_.vp8_bpred && bpred_plan(src, mbx, mby, mb_w_, h264::lambda_sad(qp), &lo, &hi)) {
                    auto at = [&](int x, int y) { return (int)ry[(size_t)y * cw_ + x]; };
                    m.ymode = kBPred;
                    set_bmodes(m, lo, hi);
                    bpred_nz = bpred_code(sy + (size_t)y0 * pitch + x0, pitch, at, mbx, mby, mb_w_, Q, lo, hi, lv, rec);
                }
                const Edge eu = edge_of(ruv, cw_, 2, 0, x0 / 2, y0 / 2, 8), ev = edge_of(ruv, cw_, 2, 1, x0 / 2, y0 / 2, 8);
                const int du = dc_of(eu, 8), dv = dc_of(ev, 8);
                best = ~0u;
                for (int mode = 0; mode < 4; ++mode) {
                    uint32_t sad = 0;
                    for (int y = 0; y < 8; ++y)
                        for (int x = 0; x < 8; ++x) {
                            const int o = (y0 / 2 + y) * pitch + (x0 + 2 * x);
                            sad += (uint32_t)std::abs((int)suv[o] - pred_px(mode, eu, 8, x, y, du));
                            sad += (uint32_t)std::abs((int)suv[o + 1] - pred_px(mode, ev, 8, x, y, dv));
                        }
                    if (sad < best) {
                        best = sad;
                        m.uvmode = (uint8_t)mode;
                    }
                }
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) {
                        cp[0][y * 8 + x] = pred_px(m.uvmode, eu, 8, x, y, du);
                        cp[1][y * 8 + x] = pred_px(m.uvmode, ev, 8, x, y, dv);
                    }
            } else {
                int mvx = 0, mvy = 0;  // quarter samples (full samples without subpel)
                h264::me_search_cpu(sy, pitch, fy, cw_, ch_, x0, y0, qp, cfg_.search_range, cfg_.subpel ? 1 : 0, &mvx,
                                    &mvy, cfg_.me_coarse);
                if (!cfg_.subpel) {  // the full-sample search's vector, as k_vp8_inter reads it
                    mvx = (mvx / 4) * 4;
                    mvy = (mvy / 4) * 4;
                }
                int lo_x, hi_x, lo_y, hi_y;
                mv_bounds(mb_w_, mb_h_, mbx, mby, &lo_x, &hi_x, &lo_y, &hi_y);
                int vx, vy;
                inter_vector(mvx, mvy, lo_x, hi_x, lo_y, hi_y, &vx, &vy);
                m.ymode = kInter;
                m.mvx = (int16_t)vx;
                m.mvy = (int16_t)vy;
                const int ix = vx >> 3, iy = vy >> 3;
                auto at_y = [&](int xx, int yy) { return (int)h264::ref_px(fy, cw_, cw_, ch_, xx, yy); };
                for (int y = 0; y < 16; ++y)
                    for (int x = 0; x < 16; ++x)
                        pred[y * 16 + x] = ((vx | vy) & 7) == 0 ? at_y(x0 + x + ix, y0 + y + iy)
                                                                 : sixtap_px(at_y, x0 + x + ix, y0 + y + iy, vx & 7, vy & 7);
                // chroma: the luma vector halved, in 1/8 chroma samples (odd full-sample luma
                // vectors land on the half-sample six-tap phase)
                const int cvx = chroma_mv(m.mvx), cvy = chroma_mv(m.mvy);
                for (int c = 0; c < 2; ++c) {
                    auto at = [&](int xx, int yy) {
                        xx = std::clamp(xx, 0, cw_ / 2 - 1);
                        yy = std::clamp(yy, 0, ch_ / 2 - 1);
                        return (int)fuv[yy * cw_ + 2 * xx + c];
                    };
                    for (int y = 0; y < 8; ++y)
                        for (int x = 0; x < 8; ++x)
                            cp[c][y * 8 + x] = sixtap_px(at, x0 / 2 + x + (cvx >> 3), y0 / 2 + y + (cvy >> 3), cvx & 7, cvy & 7);
                }
            }
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) res[y * 16 + x] = sy[(y0 + y) * pitch + x0 + x] - pred[y * 16 + x];
            for (int c = 0; c < 2; ++c)
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x)
                        cres[c][y * 8 + x] = suv[(y0 / 2 + y) * pitch + x0 + 2 * x + c] - cp[c][y * 8 + x];
            if (!key && cfg_.aq >= 3) {  // temporal class of the macroblock -> its segment (quantiser)
                const int ix = m.mvx >> 3, iy = m.mvy >> 3;
                uint32_t tsad = 0;
                for (int y = 0; y < 16; ++y)
                    for (int x = 0; x < 16; ++x)
                        tsad += (uint32_t)std::abs((int)sy[(y0 + y) * pitch + x0 + x] -
                                                   h264::ref_px(prev_src_.data(), cw_, cw_, ch_, x0 + x + ix, y0 + y + iy));
                m.seg = (uint8_t)seg_of_tclass(h264::temporal_class(tsad, m.mvx == 0 && m.mvy == 0));
            }
            const Quant Qm = m.seg ? quant_of(seg_qindex_[m.seg]) : (key ? Q : quant_of(seg_qindex_[0]));
            if (m.ymode == kBPred) {
                m.nz = bpred_nz;
                for (int k = 0; k < 16; ++k) lv[kY2 * 16 + k] = 0;
            } else {
                m.nz = code_luma16(res, pred, Qm, lv, rec);
            }
            m.nz |= code_chroma8(cres[0], cp[0], Qm, lv, crec[0], 16);
            m.nz |= code_chroma8(cres[1], cp[1], Qm, lv, crec[1], 20);
            if (!key) {  // noise-like residual that does not pay for its bits: prediction only
                uint32_t lsad = 0, bits = 0;
                long long dp = 0, dc = 0;
                for (int i = 0; i < 256; ++i) {
                    const int e = sy[(y0 + i / 16) * pitch + x0 + i % 16] - rec[i];
                    lsad += (uint32_t)std::abs(res[i]);
                    dp += res[i] * res[i];
                    dc += e * e;
                }
                m.bmodes_hi = lsad;  // the inter prediction SAD (intra_pass)
                for (int b = 0; b < 16; ++b) {
                    int n = 0;
                    for (int k = 1; k < 16; ++k) n += lv[b * 16 + k] != 0;
                    bits += vp8_block_bits(n);
                }
                int n2 = 0;
                for (int k = 0; k < 16; ++k) n2 += lv[kY2 * 16 + k] != 0;
                bits += vp8_block_bits(n2);
                if (vp8_drop_residual(lsad, dp, dc, bits, h264::lambda_sse(qp))) {
                    m.nz = 0;
                    std::memset(lv, 0, sizeof(int16_t) * kCoefPerMb);
                    for (int i = 0; i < 256; ++i) rec[i] = pred[i];
                    for (int c = 0; c < 2; ++c)
                        for (int i = 0; i < 64; ++i) crec[c][i] = cp[c][i];
                }
            }
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) ry[(y0 + y) * cw_ + x0 + x] = (uint8_t)rec[y * 16 + x];
            if (cfg_.aq >= 3)  // the next frame's previous source
                for (int y = 0; y < 16; ++y) std::memcpy(&next_src_[(size_t)(y0 + y) * cw_ + x0], sy + (y0 + y) * pitch + x0, 16);
            for (int c = 0; c < 2; ++c)
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) ruv[(y0 / 2 + y) * cw_ + x0 + 2 * x + c] = (uint8_t)crec[c][y * 8 + x];
        }
}

// Intra macroblocks in an inter frame, after every macroblock was coded inter: candidates from
// the inter reconstruction, then the candidates without a candidate causal neighbour coded intra
// (vp8_core.h vp8_intra_candidate; k_vp8_intra_cand / k_vp8_intra_code on the GPU).
void CpuVp8Encoder::intra_pass(const uint8_t* sy, const uint8_t* suv, int pitch, int qp) {
    uint8_t* ry = rec_y_[cur_].data();
    uint8_t* ruv = rec_uv_[cur_].data();
    const int lam = h264::lambda_sad(qp);
    const size_t nmb = mb_.size();
    std::vector<uint8_t> cand(nmb, 0), mode(nmb, 0);
    auto best16 = [&](int x0, int y0, int* bm) {
        const Edge e = edge_of(ry, cw_, 1, 0, x0, y0, 16);
        const int dc = dc_of(e, 16);
        uint32_t best = ~0u;
        for (int md = 0; md < 4; ++md) {
            uint32_t sad = 0;
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x)
                    sad += (uint32_t)std::abs((int)sy[(y0 + y) * pitch + x0 + x] - pred_px(md, e, 16, x, y, dc));
            if (sad < best) {
                best = sad;
                *bm = md;
            }
        }
        return best;
    };
    for (int mby = 0; mby < mb_h_; ++mby)
        for (int mbx = 0; mbx < mb_w_; ++mbx) {
            const int i = mby * mb_w_ + mbx;
            if (mb_[i].bmodes_hi <= kIntraMinSad) continue;
            int bm = 0;
            const uint32_t s = best16(mbx * 16, mby * 16, &bm);
            cand[i] = vp8_intra_candidate(mb_[i].bmodes_hi, s, lam);
            mode[i] = (uint8_t)bm;
        }
    for (int mby = 0; mby < mb_h_; ++mby)
        for (int mbx = 0; mbx < mb_w_; ++mbx) {
            const int i = mby * mb_w_ + mbx, x0 = mbx * 16, y0 = mby * 16;
            if (!cand[i] || (mbx > 0 && cand[i - 1]) || (mby > 0 && cand[i - mb_w_]) ||
                (mbx > 0 && mby > 0 && cand[i - mb_w_ - 1]))
                continue;
            Vp8Mb& m = mb_[i];
            int16_t* lv = lv_.data() + (size_t)i * kCoefPerMb;
            int pred[256], res[256], rec[256], cp[2][64], cres[2][64], crec[2][64];
            const Edge e = edge_of(ry, cw_, 1, 0, x0, y0, 16);
            const int dc = dc_of(e, 16);
            m.ymode = mode[i];
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) pred[y * 16 + x] = pred_px(m.ymode, e, 16, x, y, dc);
            const Edge eu = edge_of(ruv, cw_, 2, 0, x0 / 2, y0 / 2, 8), ev = edge_of(ruv, cw_, 2, 1, x0 / 2, y0 / 2, 8);
            const int du = dc_of(eu, 8), dv = dc_of(ev, 8);
            uint32_t best = ~0u;
            for (int md = 0; md < 4; ++md) {
                uint32_t sad = 0;
                for (int y = 0; y < 8; ++y)
                    for (int x = 0; x < 8; ++x) {
                        const int o = (y0 / 2 + y) * pitch + (x0 + 2 * x);
                        sad += (uint32_t)std::abs((int)suv[o] - pred_px(md, eu, 8, x, y, du));
                        sad += (uint32_t)std::abs((int)suv[o + 1] - pred_px(md, ev, 8, x, y, dv));
                    }
                if (sad < best) {
                    best = sad;
                    m.uvmode = (uint8_t)md;
                }
            }
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) {
                    cp[0][y * 8 + x] = pred_px(m.uvmode, eu, 8, x, y, du);
                    cp[1][y * 8 + x] = pred_px(m.uvmode, ev, 8, x, y, dv);
                }
            for (int k = 0; k < 256; ++k) res[k] = sy[(y0 + k / 16) * pitch + x0 + k % 16] - pred[k];
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 64; ++k) cres[c][k] = suv[(y0 / 2 + k / 8) * pitch + x0 + 2 * (k % 8) + c] - cp[c][k];
            const Quant Qm = quant_of(seg_qindex_[m.seg & 3]);
            m.mvx = m.mvy = 0;
            m.bmodes_hi = 0;
            m.nz = code_luma16(res, pred, Qm, lv, rec);
            m.nz |= code_chroma8(cres[0], cp[0], Qm, lv, crec[0], 16);
            m.nz |= code_chroma8(cres[1], cp[1], Qm, lv, crec[1], 20);
            for (int k = 0; k < 256; ++k) ry[(size_t)(y0 + k / 16) * cw_ + x0 + k % 16] = (uint8_t)rec[k];
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 64; ++k) ruv[(size_t)(y0 / 2 + k / 8) * cw_ + x0 + 2 * (k % 8) + c] = (uint8_t)crec[c][k];
        }
}

const std::vector<uint8_t>& CpuVp8Encoder::encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr) {
    auto run_serial = [](int n, const std::function<void(int)>& fn) {
        for (int k = 0; k < n; ++k) fn(k);
    };
    const int log2_parts = mb_h_ >= 8 ? 3 : (mb_h_ >= 4 ? 2 : (mb_h_ >= 2 ? 1 : 0));
    while (common_.wants_probe()) {  // size the first key frame, as the GPU encoder does
        const int q = common_.probe_qp();
        analyse(y, uv, pitch, true, qindex_for_qp(q), q);
        std::vector<uint8_t> tmp;
        write_frame(FrameDesc{true, cfg_.width, cfg_.height, mb_w_, mb_h_, qindex_for_qp(q), log2_parts}, mb_.data(),
                    [&](int i) { return (const int16_t*)lv_.data() + (size_t)i * kCoefPerMb; }, tmp, run_serial);
        common_.add_probe(q, (int)tmp.size());
    }
    common_.begin_frame(force_idr || !have_ref_);
    cur_ ^= 1;
    const bool key = common_.cur_idr();
    const int qindex = qindex_for_qp(common_.cur_qp());
    FrameDesc fd{key, cfg_.width, cfg_.height, mb_w_, mb_h_, qindex, log2_parts};
    fd.segmented = !key && cfg_.aq >= 3;
    for (int k = 0; k < kNumSegs; ++k) seg_qindex_[k] = qindex;
    if (fd.segmented) segment_qindices(common_.cur_qp(), cfg_.aq, seg_qindex_);
    for (int k = 0; k < kNumSegs; ++k) fd.seg_qindex[k] = seg_qindex_[k];
    lf_levels(lf_.decide(frames_, key), fd.segmented, qindex, seg_qindex_, lf_num_, fd.lf_level);
    analyse(y, uv, pitch, key, qindex, common_.cur_qp());
    if (!key && cfg_.vp8_intra) intra_pass(y, uv, pitch, common_.cur_qp());
    // the loop filter over the whole reconstruction (the next frame's reference, the decoder's output)
    if (fd.lf_level[0] | fd.lf_level[1] | fd.lf_level[2] | fd.lf_level[3])
        loop_filter_frame(rec_y_[cur_].data(), rec_uv_[cur_].data(), cw_, mb_w_, mb_h_, mb_.data(), fd.lf_level, key);
    lf_.record(frames_, key, mb_.data(), mb_w_, mb_h_);
    if (cfg_.aq >= 3) prev_src_.swap(next_src_);
    au_.clear();
    write_frame(fd, mb_.data(), [&](int i) { return (const int16_t*)lv_.data() + (size_t)i * kCoefPerMb; }, au_,
                run_serial, &tok_stats_[key ? 1 : 0][frames_ % kStatsLag]);
    ++frames_;
    int skipped = 0;
    for (const Vp8Mb& m : mb_) skipped += m.nz == 0;
    stats_.frame_index = common_.frames();
    stats_.idr = key;
    stats_.qp = common_.cur_qp();
    stats_.bytes = (int)au_.size();
    stats_.skipped_mbs = skipped;
    stats_.deblocked = (fd.lf_level[0] | fd.lf_level[1] | fd.lf_level[2] | fd.lf_level[3]) != 0;
    common_.end_frame((int)au_.size(), key);
    have_ref_ = true;
    return au_;
}

}  // namespace vp8
}  // namespace mx
