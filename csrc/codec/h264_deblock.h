// H.264 in-loop deblocking filter (ITU-T H.264 8.7) shared, __host__ __device__, by the HIP
// deblocking kernel (h264_kernels.hip k_deblock) and the CPU encoder (h264_cpu.cpp), so both
// produce bit-identical reference pictures.  NVENC filters its reconstruction in the same loop
// (`nvh264enc`, reference Dockerfile:210); the independent decoder mxdesk/codec/h264_decoder.py
// implements the same clause from the spec side and checks the result.
//
// Subset: frame macroblocks, one reference picture, disable_deblocking_filter_idc 0 with zero
// alpha / beta offsets (the slice header writes idc 0 when EncoderConfig::deblock is on, per
// picture by db_auto_decide when it is adaptive).
#pragma once
#include "h264_core.h"
#include "h264_gpu.h"

namespace mx {
namespace h264 {

// Tables 8-16 (alpha', beta' by indexA / indexB) and 8-17 (tC0' by indexA, bS = 1..3), 8-bit video.
constexpr uint8_t kDbAlpha[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   0,   0,   0,   4,   4,
                                  5,  6,  7,  8,  9,  10, 12, 13, 15,  17,  20,  22,  25,  28,  32,  36,  40,  45,
                                  50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
constexpr uint8_t kDbBeta[52] = {0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  2,  2,  2,  3,  3,  3,  3,  4,  4, 4,
                                 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
constexpr uint8_t kDbTc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1},
    {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4},
    {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11},
    {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

MXHD int db_abs(int v) { return v < 0 ? -v : v; }
MXHD int db_clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// Motion vector of raster 4x4 block `blk` (by * 4 + bx) of an inter macroblock.
MXHD void db_blk_mv(const MbInfo& m, int blk, int* mvx, int* mvy) {
    const int bx = blk & 3, by = blk >> 2;
    const bool second = (m.part == kPart16x8 && by >= 2) || (m.part == kPart8x16 && bx >= 2);
    if (m.part == kPart16x16) {
        *mvx = m.mvx;
        *mvy = m.mvy;
    } else {
        *mvx = m.pmv[second ? 2 : 0];
        *mvy = m.pmv[second ? 3 : 1];
    }
}

// Boundary strength (8.7.2.1) of the edge between raster 4x4 luma block bp of macroblock p and
// block bq of macroblock q (frame macroblocks, every inter block refers to picture 0).
MXHD int db_bs(const MbInfo& p, int bp, const MbInfo& q, int bq, bool mb_edge) {
    if (is_intra(p) || is_intra(q)) return mb_edge ? 4 : 3;
    if (p.nz_luma[bp] || q.nz_luma[bq]) return 2;
    int px, py, qx, qy;
    db_blk_mv(p, bp, &px, &py);
    db_blk_mv(q, bq, &qx, &qy);
    return (db_abs(px - qx) >= 4 || db_abs(py - qy) >= 4) ? 1 : 0;
}

// The four bS values (one per 4-sample segment) of luma edge e (0..3) of macroblock q, vertical
// (left / internal column edges) or horizontal (top / internal row edges), packed 3 bits each;
// nb = the left (vertical) or top (horizontal) macroblock for e == 0, nullptr = picture edge.
MXHD uint32_t db_edge_bs4(const MbInfo& q, const MbInfo* nb, int e, bool vertical) {
    uint32_t out = 0;
    for (int s = 0; s < 4; ++s) {
        int bs;
        if (vertical) {
            bs = e == 0 ? (nb ? db_bs(*nb, s * 4 + 3, q, s * 4, true) : 0) : db_bs(q, s * 4 + e - 1, q, s * 4 + e, false);
        } else {
            bs = e == 0 ? (nb ? db_bs(*nb, 12 + s, q, s, true) : 0) : db_bs(q, (e - 1) * 4 + s, q, e * 4 + s, false);
        }
        out |= (uint32_t)bs << (3 * s);
    }
    return out;
}

// Per-edge filter parameters: alpha, beta, tC0[bS-1] for qPav (offsets 0: indexA = indexB = qPav).
struct DbParams {
    int alpha, beta;
    uint32_t tc0;  // tC0 for bS 1, 2, 3 in bits 0..4, 5..9, 10..14 (packed: no indexed array on the GPU)
};
MXHD int db_tc0(const DbParams& d, int bs) { return (int)((d.tc0 >> (5 * (bs - 1))) & 31u); }
MXHD DbParams db_params(int qpav) {
    const int ia = db_clip3(0, 51, qpav);
    DbParams d;
    d.alpha = kDbAlpha[ia];
    d.beta = kDbBeta[ia];
    d.tc0 = (uint32_t)kDbTc0[ia][0] | ((uint32_t)kDbTc0[ia][1] << 5) | ((uint32_t)kDbTc0[ia][2] << 10);
    return d;
}

// One line of luma samples across an edge (8.7.2.3 / 8.7.2.4): p0..p2 / q0..q2 updated in place,
// p3 / q3 read only.  bS 0 leaves the line untouched.
MXHD void db_luma_line(int& p3, int& p2, int& p1, int& p0, int& q0, int& q1, int& q2, int& q3, int bs,
                       const DbParams& d) {
    const int P0 = p0, P1 = p1, P2 = p2, P3 = p3, Q0 = q0, Q1 = q1, Q2 = q2, Q3 = q3;
    if (bs == 0 || !(db_abs(P0 - Q0) < d.alpha && db_abs(P1 - P0) < d.beta && db_abs(Q1 - Q0) < d.beta)) return;
    const bool ap = db_abs(P2 - P0) < d.beta, aq = db_abs(Q2 - Q0) < d.beta;
    if (bs < 4) {
        const int tc0 = db_tc0(d, bs);
        const int tc = tc0 + (ap ? 1 : 0) + (aq ? 1 : 0);
        const int delta = db_clip3(-tc, tc, (((Q0 - P0) * 4) + (P1 - Q1) + 4) >> 3);
        p0 = clip255(P0 + delta);
        q0 = clip255(Q0 - delta);
        if (ap) p1 = P1 + db_clip3(-tc0, tc0, (P2 + ((P0 + Q0 + 1) >> 1) - (P1 * 2)) >> 1);
        if (aq) q1 = Q1 + db_clip3(-tc0, tc0, (Q2 + ((P0 + Q0 + 1) >> 1) - (Q1 * 2)) >> 1);
        return;
    }
    const bool small = db_abs(P0 - Q0) < ((d.alpha >> 2) + 2);
    if (ap && small) {
        p0 = (P2 + 2 * P1 + 2 * P0 + 2 * Q0 + Q1 + 4) >> 3;
        p1 = (P2 + P1 + P0 + Q0 + 2) >> 2;
        p2 = (2 * P3 + 3 * P2 + P1 + P0 + Q0 + 4) >> 3;
    } else {
        p0 = (2 * P1 + P0 + Q1 + 2) >> 2;
    }
    if (aq && small) {
        q0 = (P1 + 2 * P0 + 2 * Q0 + 2 * Q1 + Q2 + 4) >> 3;
        q1 = (P0 + Q0 + Q1 + Q2 + 2) >> 2;
        q2 = (2 * Q3 + 3 * Q2 + Q1 + Q0 + P0 + 4) >> 3;
    } else {
        q0 = (2 * Q1 + Q0 + P1 + 2) >> 2;
    }
}

// One line of chroma samples (chromaStyleFilteringFlag): p0 / q0 updated, p1 / q1 read only.
MXHD void db_chroma_line(int p1, int& p0, int& q0, int q1, int bs, const DbParams& d) {
    const int P0 = p0, Q0 = q0;
    if (bs == 0 || !(db_abs(P0 - Q0) < d.alpha && db_abs(p1 - P0) < d.beta && db_abs(q1 - Q0) < d.beta)) return;
    if (bs < 4) {
        const int tc = db_tc0(d, bs) + 1;
        const int delta = db_clip3(-tc, tc, (((Q0 - P0) * 4) + (p1 - q1) + 4) >> 3);
        p0 = clip255(P0 + delta);
        q0 = clip255(Q0 - delta);
        return;
    }
    p0 = (2 * p1 + P0 + q1 + 2) >> 2;
    q0 = (2 * q1 + Q0 + p1 + 2) >> 2;
}

// Adaptive in-loop filtering (EncoderConfig::deblock 2): disable_deblocking_filter_idc of a picture
// chosen from its temporal classes.  Filtering pays on moving content (sub-sample motion
// compensation of a pan or a video leaves block edges the filter smooths: +1.3 dB on the motion
// bench, profiles/r04_toolset/NOTES.md) and costs on a still desktop (it softens text and window
// edges the encoder codes exactly: -1.1 dB).  The class is taken from the coded macroblocks:
//  * moving: an inter MB with a nonzero vector;
//  * coherent: a moving MB whose vector equals its left or upper neighbour's (a pan, a scroll, a
//    moving video -- not the random vectors of noise);
//  * changed: an intra MB, or an inter MB with residual and a zero vector (text updates, cursor;
//    reported only).
// A P picture is filtered when at least half of the moving MBs move coherently and they cover
// 1/64 of the picture (flat areas of a pan keep a zero vector, so the moving share of a picture
// varies with resolution; noise moves incoherently); while the previous decision was on, a third
// and 1/128 keep it on (hysteresis: a slowing pan does not toggle the filter every frame).  An
// IDR picture keeps the previous decision.  Same integer rule in k_db_prep, k_hevc_db_auto and the
// CPU encoders.
struct DbAutoCounts {
    uint32_t coherent = 0, changed = 0, moving = 0;
};
MXHD void db_auto_count(const MbInfo* mbs, int mb_w, int i, DbAutoCounts& c) {
    const MbInfo& m = mbs[i];
    if (is_intra(m)) {
        ++c.changed;
        return;
    }
    const bool moving = m.mvx != 0 || m.mvy != 0;
    if (!moving) {
        if (m.cbp) ++c.changed;
        return;
    }
    ++c.moving;
    const int x = i % mb_w;
    auto same = [&](const MbInfo& n) { return !is_intra(n) && n.mvx == m.mvx && n.mvy == m.mvy; };
    if ((x > 0 && same(mbs[i - 1])) || (i >= mb_w && same(mbs[i - mb_w]))) ++c.coherent;
}
// The coherent count from motion vectors alone (HEVC: the 16x16 motion-search vectors of its
// units; unit i's vector at mv[i * stride], mv[i * stride + 1]).
MXHD void db_auto_count_mv(const int16_t* mv, int stride, int mb_w, int i, DbAutoCounts& c) {
    const int x = mv[(size_t)i * stride], y = mv[(size_t)i * stride + 1];
    if (x == 0 && y == 0) return;
    ++c.moving;
    auto same = [&](int j) { return mv[(size_t)j * stride] == x && mv[(size_t)j * stride + 1] == y; };
    if ((i % mb_w > 0 && same(i - 1)) || (i >= mb_w && same(i - mb_w))) ++c.coherent;
}
MXHD bool db_auto_decide(const DbAutoCounts& c, int nmb, bool prev_on) {
    // on when coherent motion is at least half of the motion and a tenth of the picture (off below
    // a twelfth once on): the 1080p pan content has 15 % coherent macroblocks and gains 1.3 dB
    // filtered, the desktop with its moving window 6.7 % and gains 0.2 dB (r06_defaults/NOTES.md)
    const uint64_t co = c.coherent;
    return co * (prev_on ? 3u : 2u) >= (uint64_t)c.moving && co * (prev_on ? 12u : 10u) >= (uint64_t)nmb && co > 0;
}

// The adaptive decision at a fixed lag (ADVICE r5 h264_encoder.cpp:696): picture n is filtered
// according to the classes of picture n - kDbLag, the newest picture whose records the host holds
// when picture n is prepared at any pipeline depth (<= 4 frames in flight), so the GPU encoder
// decides the same at depth 1 and 4 and the CPU oracle matches it frame for frame (the decision
// used to come from whichever picture had been collected last).  An IDR picture, or a lag picture
// that was an IDR, keeps the last decision.  mode: 0 off, 1 on, 2 adaptive.
constexpr int kDbLag = 4;
class DbLagDecision {
   public:
    explicit DbLagDecision(int mode = 0) : mode_(mode) {}
    void reset(int mode) { *this = DbLagDecision(mode); }
    // picture `fidx`'s filter, when it is prepared (in picture order)
    bool decide(long long fidx, bool idr) {
        if (mode_ != 2) return on_ = mode_ == 1;
        const Rec& r = ring_[(size_t)(fidx % kDbLag + kDbLag) % kDbLag];
        if (!idr && r.valid && r.fidx == fidx - kDbLag) on_ = db_auto_decide(r.c, r.nmb, on_);
        return on_;
    }
    bool on() const { return on_; }
    // picture `fidx`'s class counts, once it is coded
    void record(long long fidx, bool idr, const DbAutoCounts& c, int nmb) {
        Rec& r = ring_[(size_t)(fidx % kDbLag + kDbLag) % kDbLag];
        r.fidx = fidx;
        r.nmb = nmb;
        r.c = c;
        r.valid = !idr && mode_ == 2;
    }

   private:
    struct Rec {
        long long fidx = -1;
        int nmb = 0;
        bool valid = false;
        DbAutoCounts c;
    };
    int mode_;
    bool on_ = false;
    Rec ring_[kDbLag];
};

// QP_Y of every macroblock as a decoder sees it: the MB's own QP where it carries mb_qp_delta,
// else the predictor (the last such MB's QP in decoding order within the slice, the slice QP at
// its start).  I slices code every MB at the slice QP.
inline void db_qp_eff(const MbInfo* mbs, int nmb, int mb_w, int slice_rows, int frame_qp, bool idr, uint8_t* out) {
    const int per_slice = slice_rows * mb_w;
    int pred = frame_qp;
    for (int i = 0; i < nmb; ++i) {
        if (i % per_slice == 0) pred = frame_qp;
        if (!idr && carries_dqp(mbs[i])) pred = mbs[i].qp;
        out[i] = (uint8_t)(idr ? frame_qp : pred);
    }
}

// Serial reference: the whole picture in the order of 8.7 (per macroblock in raster order: luma
// vertical edges left to right, luma horizontal edges top to bottom, then the same for each
// chroma component).  y: luma plane, uv: interleaved chroma plane, both `pitch` wide.
inline void deblock_picture_cpu(const Geometry& g, const MbInfo* mbs, const uint8_t* qp_eff, int chroma_qp_offset,
                                uint8_t* y, uint8_t* uv, int pitch) {
    for (int mby = 0; mby < g.mb_h; ++mby)
        for (int mbx = 0; mbx < g.mb_w; ++mbx) {
            const int i = mby * g.mb_w + mbx;
            const MbInfo& q = mbs[i];
            const MbInfo* left = mbx > 0 ? &mbs[i - 1] : nullptr;
            const MbInfo* top = mby > 0 ? &mbs[i - g.mb_w] : nullptr;
            uint32_t bsv[4], bsh[4];
            for (int e = 0; e < 4; ++e) {
                bsv[e] = db_edge_bs4(q, left, e, true);
                bsh[e] = db_edge_bs4(q, top, e, false);
            }
            const int qq = qp_eff[i], ql = left ? qp_eff[i - 1] : qq, qt = top ? qp_eff[i - g.mb_w] : qq;
            const int x0 = mbx * 16, y0 = mby * 16;
            for (int dir = 0; dir < 2; ++dir) {  // 0: vertical edges, 1: horizontal edges
                for (int e = 0; e < 4; ++e) {
                    const uint32_t b4 = dir == 0 ? bsv[e] : bsh[e];
                    if (!b4) continue;
                    const DbParams d = db_params(((e == 0 ? (dir == 0 ? ql : qt) : qq) + qq + 1) >> 1);
                    for (int k = 0; k < 16; ++k) {
                        const int bs = (b4 >> (3 * (k >> 2))) & 7;
                        // sample i steps from the edge: (row, col) of p_i / q_i
                        auto at = [&](int s) -> uint8_t& {  // s = -4..3 (p3 = -4 .. q3 = 3)
                            return dir == 0 ? y[(y0 + k) * pitch + x0 + 4 * e + s] : y[(y0 + 4 * e + s) * pitch + x0 + k];
                        };
                        int p3 = at(-4), p2 = at(-3), p1 = at(-2), p0 = at(-1), q0 = at(0), q1 = at(1), q2 = at(2), q3 = at(3);
                        db_luma_line(p3, p2, p1, p0, q0, q1, q2, q3, bs, d);
                        at(-3) = (uint8_t)p2;
                        at(-2) = (uint8_t)p1;
                        at(-1) = (uint8_t)p0;
                        at(0) = (uint8_t)q0;
                        at(1) = (uint8_t)q1;
                        at(2) = (uint8_t)q2;
                    }
                }
            }
            for (int comp = 0; comp < 2; ++comp)
                for (int dir = 0; dir < 2; ++dir)
                    for (int ce = 0; ce < 2; ++ce) {  // chroma edges 0 / 4 take luma edges 0 / 8
                        const int e = 2 * ce;
                        const uint32_t b4 = dir == 0 ? bsv[e] : bsh[e];
                        if (!b4) continue;
                        const int qpp = e == 0 ? (dir == 0 ? ql : qt) : qq;
                        const DbParams d = db_params((chroma_qp(qpp, chroma_qp_offset) + chroma_qp(qq, chroma_qp_offset) + 1) >> 1);
                        const int cx0 = x0 / 2, cy0 = y0 / 2;
                        for (int k = 0; k < 8; ++k) {
                            const int bs = (b4 >> (3 * (k >> 1))) & 7;  // chroma line k = luma line 2k
                            auto at = [&](int s) -> uint8_t& {
                                return dir == 0 ? uv[(cy0 + k) * pitch + 2 * (cx0 + 4 * ce + s) + comp]
                                                : uv[(cy0 + 4 * ce + s) * pitch + 2 * (cx0 + k) + comp];
                            };
                            int p0 = at(-1), q0 = at(0);
                            db_chroma_line(at(-2), p0, q0, at(1), bs, d);
                            at(-1) = (uint8_t)p0;
                            at(0) = (uint8_t)q0;
                        }
                    }
        }
}

}  // namespace h264
}  // namespace mx
