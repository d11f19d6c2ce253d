// CPU H.264 encoder: the same decisions and arithmetic as the HIP kernels, serial.
// Serves the no-GPU plumbing configuration (BASELINE.json config 1, the reference's
// `x264enc` fallback, README.md:21) and is the bit-exact oracle for the GPU encoder.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "h264_encoder.h"
#include "h264_deblock.h"
#include "h264_mb.h"

namespace mx {
namespace h264 {

void pad_nv12(const uint8_t* y, const uint8_t* uv, int w, int h, int pitch, int coded_w, int coded_h,
              std::vector<uint8_t>& oy, std::vector<uint8_t>& ouv) {
    oy.resize((size_t)coded_w * coded_h);
    ouv.resize((size_t)coded_w * coded_h / 2);
    for (int r = 0; r < coded_h; ++r) {
        const uint8_t* s = y + (size_t)std::min(r, h - 1) * pitch;
        uint8_t* d = oy.data() + (size_t)r * coded_w;
        std::memcpy(d, s, w);
        for (int c = w; c < coded_w; ++c) d[c] = s[w - 1];
    }
    for (int r = 0; r < coded_h / 2; ++r) {
        const uint8_t* s = uv + (size_t)std::min(r, h / 2 - 1) * pitch;
        uint8_t* d = ouv.data() + (size_t)r * coded_w;
        std::memcpy(d, s, w);
        for (int c = w; c < coded_w; c += 2) {
            d[c] = s[w - 2];
            d[c + 1] = s[w - 1];
        }
    }
}

// Integer full search + quarter-pel refinement of the 16x16 block at (x0, y0): the same
// rules as k_me_full (static-block exit, cost = SAD + lambda * mv bits, tie -> shorter vector
// then lower candidate index).  Shared by the CPU H.264 and HEVC encoders.
void me_search_cpu(const uint8_t* sy, int pitch, const uint8_t* ref_y, int cw_, int ch_, int x0, int y0,
                   int frame_qp, int search_range, int subpel, int* out_mvx, int* out_mvy, int coarse) {
    const int lambda = lambda_sad(frame_qp);
    const int R = me_range(search_range);
    const int side = 2 * R + 1;
    // ---- static-block early exit, then integer full search (same rules as k_me_full)
    uint32_t sad0 = 0;
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < 16; ++k)
            sad0 += std::abs((int)sy[(y0 + r) * pitch + x0 + k] - ref_px(ref_y, cw_, cw_, ch_, x0 + k, y0 + r));
    const bool is_static = sad0 <= static_sad(frame_qp);
    unsigned long long best = ~0ull;
    auto key_of = [&](int c) {
        const int dy = c / side - R, dx = c % side - R;
        uint32_t sad = 0;
        for (int r = 0; r < 16; ++r)
            for (int k = 0; k < 16; ++k)
                sad += std::abs((int)sy[(y0 + r) * pitch + x0 + k] -
                                ref_px(ref_y, cw_, cw_, ch_, x0 + dx + k, y0 + dy + r));
        const uint32_t cost = me_cost(sad, lambda, 4 * dx, 4 * dy);
        const uint32_t dist = (uint32_t)(std::abs(dx) + std::abs(dy));
        return ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)c;
    };
    if (!is_static && coarse) {  // even-offset grid, then the 8 integer neighbours of its best
        for (int dyr = 0; dyr < side; dyr += 2)
            for (int dxr = 0; dxr < side; dxr += 2) best = std::min(best, key_of(dyr * side + dxr));
        const int cb0 = (int)(best & 0xffff), bxr = cb0 % side, byr = cb0 / side;
        unsigned long long nb = best;
        for (int k = 0; k < 8; ++k) {
            int ddx, ddy;
            subpel_offset(k, &ddx, &ddy);
            const int nxr = bxr + ddx, nyr = byr + ddy;
            if (nxr >= 0 && nxr < side && nyr >= 0 && nyr < side) nb = std::min(nb, key_of(nyr * side + nxr));
        }
        best = nb;
    }
    for (int c = 0; c < (is_static || coarse ? 0 : side * side); ++c) best = std::min(best, key_of(c));
    const int cb = (int)(best & 0xffff);
    int mvx = is_static ? 0 : 4 * ((cb % side) - R), mvy = is_static ? 0 : 4 * ((cb / side) - R);
    if (subpel && !is_static) {
        auto sad_at = [&](int vx, int vy) {
            uint32_t s = 0;
            for (int r = 0; r < 16; ++r)
                for (int k = 0; k < 16; ++k)
                    s += std::abs((int)sy[(y0 + r) * pitch + x0 + k] -
                                  luma_qpel(ref_y, cw_, cw_, ch_, (x0 + k) * 4 + vx, (y0 + r) * 4 + vy));
            return s;
        };
        uint32_t cur_cost = (uint32_t)(best >> 32);
        for (int step = 2; step >= 1; step >>= 1) {
            int bdx = 0, bdy = 0;
            uint32_t bcost = cur_cost;
            for (int k = 0; k < 8; ++k) {
                int ddx, ddy;
                subpel_offset(k, &ddx, &ddy);
                const int cx = mvx + ddx * step, cy = mvy + ddy * step;
                const uint32_t cost = me_cost(sad_at(cx, cy), lambda, cx, cy);
                if (cost < bcost) {
                    bcost = cost;
                    bdx = ddx * step;
                    bdy = ddy * step;
                }
            }
            mvx += bdx;
            mvy += bdy;
            cur_cost = bcost;
        }
    }
    *out_mvx = mvx;
    *out_mvy = mvy;
}

// Partition-aware search (the rules of k_me_full with FrameState::partitions):
//  * every integer candidate's SAD is kept per 8x8 quadrant, so one pass scores the 16x16 block
//    and the four partitions (16x8 top / bottom, 8x16 left / right), each with its own best key
//    (cost = SAD + lambda * vector bits, ties -> shorter vector, then lower candidate index);
//  * coarse mode: the even-offset grid, then the 8 integer neighbours of EACH shape's grid best;
//  * shape: 16x16 unless a partitioning's two costs + 2 lambda (mb_type ue(1) / ue(2) vs ue(0))
//    are lower (16x8 before 8x16 on ties);
//  * quarter-pel refinement (half, then quarter) of the chosen shape's vector(s), each over its
//    own rectangle.
void me_search_parts_cpu(const uint8_t* sy, int pitch, const uint8_t* ref_y, int cw_, int ch_, int x0, int y0,
                         int frame_qp, int search_range, int subpel, int coarse, MbInfo& m) {
    const int lambda = lambda_sad(frame_qp);
    const int R = me_range(search_range);
    const int side = 2 * R + 1;
    uint32_t sad0 = 0;
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < 16; ++k)
            sad0 += std::abs((int)sy[(y0 + r) * pitch + x0 + k] - ref_px(ref_y, cw_, cw_, ch_, x0 + k, y0 + r));
    m.part = kPart16x16;
    m.mvx = m.mvy = 0;
    for (int i = 0; i < 4; ++i) m.pmv[i] = 0;
    if (sad0 <= static_sad(frame_qp)) return;
    // shapes: 0 = 16x16, 1 = top, 2 = bottom, 3 = left, 4 = right (quadrants TL, TR, BL, BR)
    auto quads = [&](int c, uint32_t q[4]) {
        const int dy = c / side - R, dx = c % side - R;
        q[0] = q[1] = q[2] = q[3] = 0;
        for (int r = 0; r < 16; ++r)
            for (int k = 0; k < 16; ++k)
                q[(r >= 8 ? 2 : 0) + (k >= 8 ? 1 : 0)] += (uint32_t)std::abs(
                    (int)sy[(y0 + r) * pitch + x0 + k] - ref_px(ref_y, cw_, cw_, ch_, x0 + dx + k, y0 + dy + r));
    };
    auto shape_sad = [](const uint32_t q[4], int s) {
        switch (s) {
            case 0: return q[0] + q[1] + q[2] + q[3];
            case 1: return q[0] + q[1];
            case 2: return q[2] + q[3];
            case 3: return q[0] + q[2];
            default: return q[1] + q[3];
        }
    };
    auto key = [&](uint32_t sad, int c) {
        const int dy = c / side - R, dx = c % side - R;
        const uint32_t cost = me_cost(sad, lambda, 4 * dx, 4 * dy);
        const uint32_t dist = (uint32_t)(std::abs(dx) + std::abs(dy));
        return ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)c;
    };
    unsigned long long best[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    auto visit = [&](int c, unsigned long long* b) {
        uint32_t q[4];
        quads(c, q);
        for (int s = 0; s < 5; ++s) b[s] = std::min(b[s], key(shape_sad(q, s), c));
    };
    if (coarse) {
        for (int dyr = 0; dyr < side; dyr += 2)
            for (int dxr = 0; dxr < side; dxr += 2) visit(dyr * side + dxr, best);
        unsigned long long nb[5];
        for (int s = 0; s < 5; ++s) nb[s] = best[s];
        for (int s = 0; s < 5; ++s) {
            const int cb0 = (int)(best[s] & 0xffff), bxr = cb0 % side, byr = cb0 / side;
            for (int k = 0; k < 8; ++k) {
                int ddx, ddy;
                subpel_offset(k, &ddx, &ddy);
                const int nxr = bxr + ddx, nyr = byr + ddy;
                if (nxr < 0 || nxr >= side || nyr < 0 || nyr >= side) continue;
                uint32_t q[4];
                quads(nyr * side + nxr, q);
                nb[s] = std::min(nb[s], key(shape_sad(q, s), nyr * side + nxr));
            }
        }
        for (int s = 0; s < 5; ++s) best[s] = nb[s];
    } else {
        for (int c = 0; c < side * side; ++c) visit(c, best);
    }
    auto cost_of = [](unsigned long long k) { return (uint32_t)(k >> 32); };
    const uint32_t c16 = cost_of(best[0]);
    const uint32_t ch = cost_of(best[1]) + cost_of(best[2]) + 2u * (uint32_t)lambda;
    const uint32_t cv = cost_of(best[3]) + cost_of(best[4]) + 2u * (uint32_t)lambda;
    const int part = (c16 <= ch && c16 <= cv) ? kPart16x16 : (ch <= cv ? kPart16x8 : kPart8x16);
    // rectangle of each shape (x, y, w, h) and the refinement
    constexpr int kRect[5][4] = {{0, 0, 16, 16}, {0, 0, 16, 8}, {0, 8, 16, 8}, {0, 0, 8, 16}, {8, 0, 8, 16}};
    auto refine = [&](int s, int* vx, int* vy) {
        const int cb = (int)(best[s] & 0xffff);
        *vx = 4 * ((cb % side) - R);
        *vy = 4 * ((cb / side) - R);
        if (!subpel) return;
        const int rx = kRect[s][0], ry = kRect[s][1], rw = kRect[s][2], rh = kRect[s][3];
        auto sad_at = [&](int cx, int cy) {
            uint32_t t = 0;
            for (int r = ry; r < ry + rh; ++r)
                for (int k = rx; k < rx + rw; ++k)
                    t += std::abs((int)sy[(y0 + r) * pitch + x0 + k] -
                                  luma_qpel(ref_y, cw_, cw_, ch_, (x0 + k) * 4 + cx, (y0 + r) * 4 + cy));
            return t;
        };
        uint32_t cur = cost_of(best[s]);
        for (int step = 2; step >= 1; step >>= 1) {
            int bdx = 0, bdy = 0;
            uint32_t bcost = cur;
            for (int k = 0; k < 8; ++k) {
                int ddx, ddy;
                subpel_offset(k, &ddx, &ddy);
                const int cx = *vx + ddx * step, cy = *vy + ddy * step;
                const uint32_t cost = me_cost(sad_at(cx, cy), lambda, cx, cy);
                if (cost < bcost) {
                    bcost = cost;
                    bdx = ddx * step;
                    bdy = ddy * step;
                }
            }
            *vx += bdx;
            *vy += bdy;
            cur = bcost;
        }
    };
    int vx, vy;
    if (part == kPart16x16) {
        refine(0, &vx, &vy);
        m.mvx = (int16_t)vx;
        m.mvy = (int16_t)vy;
        return;
    }
    const int cb = (int)(best[0] & 0xffff);  // the 16x16 vector stays integer here
    m.mvx = (int16_t)(4 * ((cb % side) - R));
    m.mvy = (int16_t)(4 * ((cb / side) - R));
    m.part = (uint8_t)part;
    const int s0 = part == kPart16x8 ? 1 : 3;
    for (int i = 0; i < 2; ++i) {
        refine(s0 + i, &vx, &vy);
        m.pmv[2 * i] = (int16_t)vx;
        m.pmv[2 * i + 1] = (int16_t)vy;
    }
}

CpuH264Encoder::CpuH264Encoder(const EncoderConfig& cfg) : cfg_(cfg.with_aq_default(4)), common_(cfg) {
    db_lag_.reset(cfg_.h264_deblock_mode());
    cw_ = common_.mb_w() * 16;
    ch_ = common_.mb_h() * 16;
    for (int i = 0; i < 2; ++i) {
        rec_y_[i].assign((size_t)cw_ * ch_, 16);
        rec_uv_[i].assign((size_t)cw_ * ch_ / 2, 128);
    }
    mb_.resize((size_t)common_.mb_w() * common_.mb_h());
    coef_.resize(mb_.size() * kCoefStride);
}

static Geometry geom_of(const EncoderCommon& c, int cw, int ch) {
    Geometry g;
    g.width = c.config().width;
    g.height = c.config().height;
    g.mb_w = c.mb_w();
    g.mb_h = c.mb_h();
    g.coded_w = cw;
    g.coded_h = ch;
    g.pitch = cw;
    return g;
}

// Open-loop intra analysis of one macroblock (source neighbours): the same costs and decision
// as k_intra_analyze.
static IntraDecision analyze_intra_mb(const Geometry& g, const uint8_t* sy, const uint8_t* suv, int pitch, int mbx,
                                      int mby, int slice_rows, int qp, bool allow4) {
    const Avail av = mb_avail(g, mbx, mby, slice_rows);
    const int x0 = mbx * 16, y0 = mby * 16;
    IntraCosts c;
    for (int b = 0; b < 16; ++b)
        for (int m = 0; m < 9; ++m) c.c4[b][m] = i4_cost(sy, pitch, x0, y0, b, m, av.left, av.top, av.topright, av.topleft);
    const NbMb nl = nbmb_from_plane(sy, pitch, x0, y0, 16, 1, 0, av.left, av.top, av.topleft);
    for (int m = 0; m < 4; ++m) {
        if (!i16_mode_ok(m, nl)) {
            c.c16[m] = kCostInf;
            continue;
        }
        const PredMb p = prep_i16(m, nl);
        uint32_t t = 0;
        for (int rb = 0; rb < 16; ++rb) t += i16_block_cost(sy, pitch, x0, y0, rb, p, nl);
        c.c16[m] = t;
    }
    for (int m = 0; m < 4; ++m) {
        uint32_t t = 0;
        for (int comp = 0; comp < 2; ++comp) {
            const NbMb nc = nbmb_from_plane(suv, pitch, x0 / 2, y0 / 2, 8, 2, comp, av.left, av.top, av.topleft);
            if (!chroma_mode_ok(m, nc)) {
                t = kCostInf;
                break;
            }
            const PredMb p = prep_chroma(m, nc);
            for (int cb = 0; cb < 4; ++cb) t += chroma_block_cost(suv, pitch, x0 / 2, y0 / 2, comp, cb, p, nc);
        }
        c.cc[m] = t;
    }
    return decide_intra(c, qp, allow4);
}

static void set_intra(MbInfo& m, const IntraDecision& d, int qp) {
    m.type = (uint8_t)d.type;
    m.i16_mode = (uint8_t)d.i16_mode;
    m.chroma_mode = (uint8_t)d.chroma_mode;
    for (int rb = 0; rb < 16; ++rb) i4_set(m.i4, rb, d.i4[rb]);
    m.qp = (uint8_t)qp;
    m.mvx = 0;
    m.mvy = 0;
}

// Closed-loop coding of one intra macroblock (modes already decided): prediction from the
// reconstruction, transform, quantisation, reconstruction; the same arithmetic as k_intra_wave.
static void code_intra_mb(const Geometry& g, const uint8_t* sy, const uint8_t* suv, int pitch, uint8_t* rec_y,
                          uint8_t* rec_uv, int cw, int mbx, int mby, int slice_rows, int qp, int chroma_qp_offset,
                          MbInfo& m, int16_t* mc) {
    const Avail av = mb_avail(g, mbx, mby, slice_rows);
    const int x0 = mbx * 16, y0 = mby * 16;
    const int qpc = chroma_qp(qp, chroma_qp_offset);
    int cbp_l = 0;
    if (m.type == kMbI4x4) {
        for (int b = 0; b < 16; ++b) {
            const int bx = kBlkX[b], by = kBlkY[b];
            const Nb4 n = nb4_from_plane(rec_y, cw, x0, y0, bx, by, av.left, av.top, av.topright, av.topleft);
            const int mode = i4_get(m.i4, by * 4 + bx);
            int pred[16], x[16], y[16], z[16], d[16], r[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    pred[i * 4 + j] = pred4x4_px(mode, n, j, i);
                    x[i * 4 + j] = sy[(y0 + 4 * by + i) * pitch + x0 + 4 * bx + j] - pred[i * 4 + j];
                }
            fdct4x4(x, y);
            const int nz = quant4x4(y, z, qp, true, 0);
            for (int k = 0; k < 16; ++k) mc[kCoefLuma + b * 16 + k] = (int16_t)z[kZigzag4x4[k]];
            dequant4x4(z, d, qp, 0);
            idct4x4(d, r);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    rec_y[(y0 + 4 * by + i) * cw + x0 + 4 * bx + j] = (uint8_t)clip255(pred[i * 4 + j] + r[i * 4 + j]);
            m.nz_luma[by * 4 + bx] = (uint8_t)nz;
            if (nz) cbp_l |= 1 << (b >> 2);
        }
    } else {  // Intra16x16
        const NbMb n = nbmb_from_plane(rec_y, cw, x0, y0, 16, 1, 0, av.left, av.top, av.topleft);
        const PredMb p = prep_i16(m.i16_mode, n);
        int z[16][16], ldc[16], nzl[16];
        bool luma_ac = false;
        for (int b = 0; b < 16; ++b) {
            const int bx = kBlkX[b], by = kBlkY[b];
            int x[16], y[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    x[i * 4 + j] = sy[(y0 + 4 * by + i) * pitch + x0 + 4 * bx + j] - pred16_px(p, n, 4 * bx + j, 4 * by + i);
            fdct4x4(x, y);
            ldc[by * 4 + bx] = y[0];
            nzl[b] = quant4x4(y, z[b], qp, true, 1);
            luma_ac |= nzl[b] > 0;
            for (int k = 1; k < 16; ++k) mc[kCoefLuma + b * 16 + k] = (int16_t)z[b][kZigzag4x4[k]];
            mc[kCoefLuma + b * 16] = 0;
        }
        int zd[16], dq[16];
        quant_dc_luma(ldc, zd, qp);
        for (int k = 0; k < 16; ++k) mc[kCoefLumaDc + k] = (int16_t)zd[kZigzag4x4[k]];
        dequant_dc_luma(zd, dq, qp);
        for (int b = 0; b < 16; ++b) {
            const int bx = kBlkX[b], by = kBlkY[b];
            int d[16], rr[16];
            if (luma_ac)
                dequant4x4(z[b], d, qp, 1);
            else
                for (int i = 1; i < 16; ++i) d[i] = 0;
            d[0] = dq[by * 4 + bx];
            idct4x4(d, rr);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    rec_y[(y0 + 4 * by + i) * cw + x0 + 4 * bx + j] =
                        (uint8_t)clip255(pred16_px(p, n, 4 * bx + j, 4 * by + i) + rr[i * 4 + j]);
            m.nz_luma[by * 4 + bx] = (uint8_t)(luma_ac ? nzl[b] : 0);
        }
        cbp_l = luma_ac ? 15 : 0;
    }
    bool any_ac = false, any_dc = false;
    for (int comp = 0; comp < 2; ++comp) {
        const NbMb n = nbmb_from_plane(rec_uv, cw, x0 / 2, y0 / 2, 8, 2, comp, av.left, av.top, av.topleft);
        const PredMb p = prep_chroma(m.chroma_mode, n);
        int zc[4][16], dcin[4];
        for (int cbk = 0; cbk < 4; ++cbk) {
            const int bx = cbk & 1, by = cbk >> 1;
            int x[16], y[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    x[i * 4 + j] = suv[(y0 / 2 + 4 * by + i) * pitch + 2 * (x0 / 2 + 4 * bx + j) + comp] -
                                   predc_px(p, n, 4 * bx + j, 4 * by + i);
            fdct4x4(x, y);
            dcin[cbk] = y[0];
            const int nz = quant4x4(y, zc[cbk], qpc, true, 1);
            for (int k = 1; k < 16; ++k) mc[kCoefChromaAc + (comp * 4 + cbk) * 16 + k] = (int16_t)zc[cbk][kZigzag4x4[k]];
            (comp ? m.nz_cr : m.nz_cb)[cbk] = (uint8_t)nz;
            any_ac |= nz > 0;
        }
        int zdc[4], dqc[4];
        any_dc |= quant_dc_chroma(dcin, zdc, qpc, true) > 0;
        for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + comp * 4 + i] = (int16_t)zdc[i];
        dequant_dc_chroma(zdc, dqc, qpc);
        for (int cbk = 0; cbk < 4; ++cbk) {
            const int bx = cbk & 1, by = cbk >> 1;
            int d[16], rr[16];
            dequant4x4(zc[cbk], d, qpc, 1);
            d[0] = dqc[cbk];
            idct4x4(d, rr);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    rec_uv[(y0 / 2 + 4 * by + i) * cw + 2 * (x0 / 2 + 4 * bx + j) + comp] =
                        (uint8_t)clip255(predc_px(p, n, 4 * bx + j, 4 * by + i) + rr[i * 4 + j]);
        }
    }
    m.cbp = (uint8_t)(cbp_l | ((any_ac ? 2 : (any_dc ? 1 : 0)) << 4));
}

void CpuH264Encoder::encode_inter(const uint8_t* sy, const uint8_t* suv, int pitch) {
    const Geometry g = geom_of(common_, cw_, ch_);
    const uint8_t* ref_y = rec_y_[cur_ ^ 1].data();
    const uint8_t* ref_uv = rec_uv_[cur_ ^ 1].data();
    // the motion search reads the reference before its in-loop filter (the GPU encoder searches
    // beside k_deblock); prediction uses the filtered reference
    const uint8_t* me_ref = ref_deblocked_ ? rec_unf_y_.data() : ref_y;
    uint8_t* rec_y = rec_y_[cur_].data();
    uint8_t* rec_uv = rec_uv_[cur_].data();
    const int frame_qp = frame_qp_();
    for (int mby = 0; mby < g.mb_h; ++mby)
        for (int mbx = 0; mbx < g.mb_w; ++mbx) {
            const int mbi = mby * g.mb_w + mbx, x0 = mbx * 16, y0 = mby * 16;
            MbInfo& m = mb_[mbi];
            std::memset(&m, 0, sizeof m);
            if (cfg_.partitions) {
                me_search_parts_cpu(sy, pitch, me_ref, cw_, ch_, x0, y0, frame_qp, cfg_.search_range, cfg_.subpel,
                                    cfg_.me_coarse, m);
            } else {
                int vx = 0, vy = 0;
                me_search_cpu(sy, pitch, me_ref, cw_, ch_, x0, y0, frame_qp, cfg_.search_range, cfg_.subpel, &vx, &vy,
                              cfg_.me_coarse);
                m.mvx = (int16_t)vx;
                m.mvy = (int16_t)vy;
            }
            m.type = kMbP16x16;
            // ---- prediction + residual (per partition: each sample's vector)
            int pred[384], res[384];
            uint32_t lsad = 0;
            for (int r = 0; r < 16; ++r)
                for (int k = 0; k < 16; ++k) {
                    const Mv v = px_mv(m, k, r);
                    const int p = luma_qpel(ref_y, cw_, cw_, ch_, (x0 + k) * 4 + v.x, (y0 + r) * 4 + v.y);
                    pred[r * 16 + k] = p;
                    res[r * 16 + k] = sy[(y0 + r) * pitch + x0 + k] - p;
                    lsad += (uint32_t)std::abs(res[r * 16 + k]);
                }
            // temporal class: the source's change against the previous source, displaced by the
            // integer part of each sample's vector (aq 3)
            uint32_t tsad = 0;
            bool zero_mv = true;
            if (cfg_.aq >= 3 && !prev_src_.empty()) {
                for (int r = 0; r < 16; ++r)
                    for (int k = 0; k < 16; ++k) {
                        const Mv v = px_mv(m, k, r);
                        zero_mv = zero_mv && v.x == 0 && v.y == 0;
                        tsad += (uint32_t)std::abs((int)sy[(y0 + r) * pitch + x0 + k] -
                                                   (int)ref_px(prev_src_.data(), cw_, cw_, ch_, x0 + k + (v.x >> 2),
                                                               y0 + r + (v.y >> 2)));
                    }
            }
            const int tcls = temporal_class(tsad, zero_mv);
            const int qp = mb_qp_for(frame_qp, lsad, tcls, cfg_.aq);
            const int qpc = chroma_qp(qp, cfg_.chroma_qp_offset);
            m.qp = (uint8_t)qp;
            for (int comp = 0; comp < 2; ++comp)
                for (int r = 0; r < 8; ++r)
                    for (int k = 0; k < 8; ++k) {
                        const int xc = x0 / 2 + k, yc = y0 / 2 + r;
                        const Mv v = px_mv(m, 2 * k, 2 * r);
                        const int p = chroma_pred8(ref_uv, cw_, cw_ / 2, ch_ / 2, comp, xc * 8 + v.x, yc * 8 + v.y);
                        pred[256 + comp * 64 + r * 8 + k] = p;
                        res[256 + comp * 64 + r * 8 + k] = suv[yc * pitch + 2 * xc + comp] - p;
                    }
            int16_t* mc = coef_.data() + (size_t)mbi * kCoefStride;
            int cbp = 0;
            uint32_t satd = 0;
            int zsb[16][16], rrb[16][16], nzb[16];
            long long d_pred = 0, d_coded = 0;
            uint32_t bits = 0;
            for (int b = 0; b < 16; ++b) {
                const int bx = kBlkX[b], by = kBlkY[b];
                int x[16];
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[(by * 4 + i) * 16 + bx * 4 + j];
                satd += satd4x4(x);
                nzb[b] = luma_block_inter(x, qp, zsb[b], rrb[b]);
                bits += block_bits_est(nzb[b]);
                for (int i = 0; i < 16; ++i) {
                    const int pv = pred[(by * 4 + (i >> 2)) * 16 + bx * 4 + (i & 3)];
                    const int e = pv + x[i] - clip255(pv + rrb[b][i]);
                    d_pred += x[i] * x[i];
                    d_coded += e * e;
                }
            }
            const bool drop = drop_luma_for(cfg_.aq, lsad, tcls, qp, d_pred, d_coded, bits);
            for (int b = 0; b < 16; ++b) {
                const int bx = kBlkX[b], by = kBlkY[b];
                const int nz = drop ? 0 : nzb[b];
                for (int k = 0; k < 16; ++k) mc[kCoefLuma + b * 16 + k] = (int16_t)(drop ? 0 : zsb[b][k]);
                m.nz_luma[by * 4 + bx] = (uint8_t)nz;
                if (nz) cbp |= 1 << (b >> 2);
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j)
                        rec_y[(y0 + by * 4 + i) * cw_ + x0 + bx * 4 + j] = (uint8_t)clip255(
                            pred[(by * 4 + i) * 16 + bx * 4 + j] + (drop ? 0 : rrb[b][i * 4 + j]));
            }
            if (drop_chroma_for(cfg_.aq, tcls, drop))  // chroma residual goes with the luma decision
                for (int i = 256; i < 384; ++i) res[i] = 0;
            bool any_ac = false, any_dc = false;
            for (int comp = 0; comp < 2; ++comp) {
                int z[4][16], dcin[4];
                for (int cbk = 0; cbk < 4; ++cbk) {
                    const int bx = cbk & 1, by = cbk >> 1;
                    int x[16], y[16];
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j];
                    fdct4x4(x, y);
                    dcin[cbk] = y[0];
                    const int nz = quant4x4(y, z[cbk], qpc, false, 1);
                    for (int k = 1; k < 16; ++k)
                        mc[kCoefChromaAc + (comp * 4 + cbk) * 16 + k] = (int16_t)z[cbk][kZigzag4x4[k]];
                    (comp ? m.nz_cr : m.nz_cb)[cbk] = (uint8_t)nz;
                    any_ac |= nz > 0;
                }
                int zd[4], dq[4];
                any_dc |= quant_dc_chroma(dcin, zd, qpc, false) > 0;
                for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + comp * 4 + i] = (int16_t)zd[i];
                dequant_dc_chroma(zd, dq, qpc);
                for (int cbk = 0; cbk < 4; ++cbk) {
                    const int bx = cbk & 1, by = cbk >> 1;
                    int d[16], rr[16];
                    dequant4x4(z[cbk], d, qpc, 1);
                    d[0] = dq[cbk];
                    idct4x4(d, rr);
                    const int xc = x0 / 2 + bx * 4, yc = y0 / 2 + by * 4;
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j < 4; ++j)
                            rec_uv[(yc + i) * cw_ + 2 * (xc + j) + comp] = (uint8_t)clip255(
                                pred[256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j] + rr[i * 4 + j]);
                }
            }
            cbp |= (any_ac ? 2 : (any_dc ? 1 : 0)) << 4;
            m.cbp = (uint8_t)cbp;
            m.cost = inter_cost_mb(satd, frame_qp, m);
        }
    // intra macroblocks in the P slice: open-loop decision against the inter cost, local-maximum
    // selection (independent intra MBs), then their coding from the final inter reconstruction
    // (the same selection and arithmetic as k_intra_analyze + k_intra_p)
    if (!cfg_.intra_in_p) return;
    const int nmb = g.mb_w * g.mb_h;
    std::vector<int32_t> gain(nmb, 0);
    std::vector<IntraDecision> dec(nmb);
    for (int mbi = 0; mbi < nmb; ++mbi) {
        if (!intra_candidate(mb_[mbi].cost)) continue;
        dec[mbi] = analyze_intra_mb(g, sy, suv, pitch, mbi % g.mb_w, mbi / g.mb_w, g.mb_h, frame_qp, cfg_.intra4x4 != 0);
        gain[mbi] = intra_gain(dec[mbi].cost_luma, mb_[mbi].cost, frame_qp);
    }
    for (int mbi = 0; mbi < nmb; ++mbi)
        if (intra_selected(gain.data(), g.mb_w, g.mb_h, mbi % g.mb_w, mbi / g.mb_w)) set_intra(mb_[mbi], dec[mbi], frame_qp);
    for (int mbi = 0; mbi < nmb; ++mbi)
        if (is_intra(mb_[mbi]))
            code_intra_mb(g, sy, suv, pitch, rec_y, rec_uv, cw_, mbi % g.mb_w, mbi / g.mb_w, g.mb_h, mb_[mbi].qp,
                          cfg_.chroma_qp_offset, mb_[mbi], coef_.data() + (size_t)mbi * kCoefStride);
}

void CpuH264Encoder::encode_intra(const uint8_t* sy, const uint8_t* suv, int pitch) {
    const Geometry g = geom_of(common_, cw_, ch_);
    uint8_t* rec_y = rec_y_[cur_].data();
    uint8_t* rec_uv = rec_uv_[cur_].data();
    const int qp = frame_qp_();
    const int rows = idr_slice_rows(g.mb_h);
    for (int mbi = 0; mbi < g.mb_w * g.mb_h; ++mbi) {
        MbInfo& m = mb_[mbi];
        std::memset(&m, 0, sizeof m);
        set_intra(m, analyze_intra_mb(g, sy, suv, pitch, mbi % g.mb_w, mbi / g.mb_w, rows, qp, cfg_.intra4x4 != 0), qp);
    }
    for (int mbi = 0; mbi < g.mb_w * g.mb_h; ++mbi)
        code_intra_mb(g, sy, suv, pitch, rec_y, rec_uv, cw_, mbi % g.mb_w, mbi / g.mb_w, rows, qp, cfg_.chroma_qp_offset,
                      mb_[mbi], coef_.data() + (size_t)mbi * kCoefStride);
}

void CpuH264Encoder::decide_deblock() { deblock_now_ = db_lag_.decide((long long)enc_seq_, common_.cur_idr()); }

void CpuH264Encoder::update_deblock_decision() {
    db_counts_ = DbAutoCounts{};
    const Geometry g = geom_of(common_, cw_, ch_);
    if (!common_.cur_idr())  // an IDR picture's record is invalid: its lag picture keeps the decision
        for (int i = 0; i < g.mb_w * g.mb_h; ++i) db_auto_count(mb_.data(), g.mb_w, i, db_counts_);
    db_lag_.record((long long)enc_seq_, common_.cur_idr(), db_counts_, g.mb_w * g.mb_h);
}

void CpuH264Encoder::entropy(std::vector<uint8_t>& payload, std::vector<uint32_t>& soff, std::vector<uint32_t>& slen) {
    const Geometry g = geom_of(common_, cw_, ch_);
    const bool idr = common_.cur_idr();
    const int slice_rows = idr ? idr_slice_rows(g.mb_h) : g.mb_h;
    const int per_slice = slice_rows * g.mb_w;
    const int nmb = g.mb_w * g.mb_h;
    std::vector<uint32_t> words((size_t)nmb * kSlotWords / 4 + 4096);
    mb_bits_.assign(nmb, 0);
    for (int first = 0; first < nmb; first += per_slice) {
        const int last = std::min(first + per_slice, nmb);
        BitWriter w;
        w.init(words.data());
        write_slice_header(w, make_slice_params(first, idr, common_.cur_frame_num(), common_.log2_max_frame_num(),
                                                common_.cur_idr_pic_id(), frame_qp_() - common_.pic_init_qp(),
                                                deblock_now_ ? 0 : 1));
        int run = 0;
        int qp_pred = frame_qp_();  // mb_qp_delta predictor: QP of the last MB that carried one
        for (int mbi = first; mbi < last; ++mbi) {
            const Avail av = mb_avail(g, mbi % g.mb_w, mbi / g.mb_w, slice_rows);
            int mvd[4];
            const MbNbrs nb = mb_nbrs(mb_.data(), mbi, g.mb_w);
            const bool skip = decide_skip(nb, av, mvd);
            mb_[mbi].skip = skip;
            if (skip) {
                ++run;
                continue;
            }
            const uint32_t b0 = w.bits;
            if (!idr) {
                put_ue(w, (uint32_t)run);
                run = 0;
            }
            const int16_t* mc = coef_.data() + (size_t)mbi * kCoefStride;
            int dqp = 0;
            if (!idr && carries_dqp(mb_[mbi])) {
                dqp = qp_delta(mb_[mbi].qp, qp_pred);
                qp_pred = mb_[mbi].qp;
            }
            for (int role = 0; role < kNumRoles; ++role)
                code_role(w, role, g, idr, nb, mc, av, mvd, dqp);
            mb_bits_[mbi] = w.bits - b0;
        }
        if (!idr && run > 0) put_ue(w, (uint32_t)run);
        w.put(1, 1);
        w.flush();
        soff.push_back((uint32_t)payload.size());
        const uint32_t nbytes = (w.bits + 7) / 8;
        for (uint32_t i = 0; i < nbytes; ++i) payload.push_back((uint8_t)(words[i / 4] >> (24 - 8 * (i % 4))));
        slen.push_back(nbytes);
    }
}

const std::vector<uint8_t>& CpuH264Encoder::encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr) {
    while (common_.wants_probe()) {  // size the first IDR (rate control), as the GPU encoder does
        qp_override_ = common_.probe_qp();
        encode_intra(y, uv, pitch);
        std::vector<uint8_t> payload;
        std::vector<uint32_t> soff, slen;
        entropy(payload, soff, slen);
        common_.add_probe(qp_override_, (int)(payload.size() + soff.size() * 6 + 32));
        qp_override_ = -1;
    }
    common_.begin_frame(force_idr || !have_ref_);
    cur_ ^= 1;
    ++enc_seq_;
    // this frame's source becomes the previous source of the next one (temporal AQ classes)
    struct SaveSrc {
        std::vector<uint8_t>& d;
        const uint8_t* y;
        int pitch, cw, ch;
        ~SaveSrc() {
            d.resize((size_t)cw * ch);
            for (int r = 0; r < ch; ++r) std::memcpy(d.data() + (size_t)r * cw, y + (size_t)r * pitch, cw);
        }
    } save_src{prev_src_, y, pitch, cw_, ch_};
    if (common_.cur_idr())
        encode_intra(y, uv, pitch);
    else
        encode_inter(y, uv, pitch);
    decide_deblock();
    std::vector<uint8_t> payload;
    std::vector<uint32_t> soff, slen;
    entropy(payload, soff, slen);
    if (deblock_now_) {  // in-loop filter: the next picture predicts from the filtered one
        rec_unf_y_ = rec_y_[cur_];  // and searches the unfiltered one
        const Geometry g = geom_of(common_, cw_, ch_);
        std::vector<uint8_t> qpe(mb_.size());
        db_qp_eff(mb_.data(), (int)mb_.size(), g.mb_w, common_.cur_idr() ? idr_slice_rows(g.mb_h) : g.mb_h,
                  frame_qp_(), common_.cur_idr(), qpe.data());
        deblock_picture_cpu(g, mb_.data(), qpe.data(), cfg_.chroma_qp_offset, rec_y_[cur_].data(), rec_uv_[cur_].data(),
                            cw_);
    }
    update_deblock_decision();
    ref_deblocked_ = deblock_now_;
    au_.clear();
    if (common_.cur_idr()) common_.write_parameter_sets(au_);
    int skipped = 0;
    for (const MbInfo& m : mb_) skipped += m.skip;
    for (size_t s = 0; s < soff.size(); ++s)
        common_.write_slice_nal(au_, payload.data() + soff[s], slen[s], common_.cur_idr());
    stats_.frame_index = common_.frames();
    stats_.idr = common_.cur_idr();
    stats_.qp = common_.cur_qp();
    stats_.bytes = (int)au_.size();
    stats_.skipped_mbs = skipped;
    stats_.deblocked = deblock_now_ ? 1 : 0;
    stats_.db_coherent = (int)db_counts_.coherent;
    stats_.db_changed = (int)db_counts_.changed;
    stats_.db_moving = (int)db_counts_.moving;
    common_.end_frame((int)au_.size(), common_.cur_idr());
    have_ref_ = true;
    return au_;
}

}  // namespace h264
}  // namespace mx
