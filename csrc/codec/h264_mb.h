// Macroblock-level syntax helpers shared by the HIP kernels and the CPU encoder:
// neighbour availability, nC prediction, motion-vector prediction / P_Skip decision and
// the per-"role" CAVLC coding of one macroblock (role 0 = header, 1 = Intra16x16 DC,
// 2..17 = luma 4x4 blocks in blkIdx order, 18/19 = chroma DC, 20..27 = chroma AC).
// Coding roles in ascending order reproduces macroblock_layer() syntax order.
#pragma once
#include "h264_core.h"
#include "h264_gpu.h"
#include "h264_intra.h"

namespace mx {
namespace h264 {

constexpr int kNumRoles = 28;

struct Avail {
    bool left, top, topright, topleft;
};

MXHD Avail mb_avail(const Geometry& g, int mbx, int mby, int slice_rows) {
    Avail a;
    const bool top_same_slice = mby > 0 && (mby / slice_rows) == ((mby - 1) / slice_rows);
    a.left = mbx > 0;
    a.top = top_same_slice;
    a.topright = top_same_slice && mbx < g.mb_w - 1;
    a.topleft = top_same_slice && mbx > 0;
    return a;
}

MXHD int combine_nc(bool ha, int na, bool hb, int nb) {
    if (ha && hb) return (na + nb + 1) >> 1;
    if (ha) return na;
    if (hb) return nb;
    return 0;
}

// A macroblock and its neighbours (left, top, top-right, top-left) as the entropy coder reads
// them: pointers into the frame's MbInfo array (CPU) or into LDS copies (k_cavlc).  A pointer
// is only dereferenced when the neighbour is available.
struct MbNbrs {
    const MbInfo* self;
    const MbInfo* left;
    const MbInfo* top;
    const MbInfo* topright;
    const MbInfo* topleft;
};
MXHD MbNbrs mb_nbrs(const MbInfo* mbs, int mbi, int mb_w) {
    return MbNbrs{&mbs[mbi], &mbs[mbi - 1], &mbs[mbi - mb_w], &mbs[mbi - mb_w + 1], &mbs[mbi - mb_w - 1]};
}

// Vector of 4x4 block (bx, by) of an inter macroblock (partition-aware).
MXHD Mv blk_mv(const MbInfo& m, int bx, int by) {
    if (m.part == kPart16x8) return by < 2 ? Mv{m.pmv[0], m.pmv[1]} : Mv{m.pmv[2], m.pmv[3]};
    if (m.part == kPart8x16) return bx < 2 ? Mv{m.pmv[0], m.pmv[1]} : Mv{m.pmv[2], m.pmv[3]};
    return Mv{m.mvx, m.mvy};
}
// Vector of luma sample (x, y) of the macroblock.
MXHD Mv px_mv(const MbInfo& m, int x, int y) { return blk_mv(m, x >> 2, y >> 2); }

// Neighbour for motion-vector prediction: block (bx, by) of macroblock p.
MXHD MvNb mv_nb_blk(const MbInfo* p, bool avail, int bx, int by) {
    MvNb n;
    n.avail = avail;
    n.ref = -1;
    n.mv = Mv{0, 0};
    if (!avail) return n;
    const MbInfo& m = *p;
    if (m.type == kMbP16x16) {
        n.ref = 0;
        n.mv = blk_mv(m, bx, by);
    }
    return n;
}

// 8.4.1.3 prediction of partition `idx` (0 / 1) of a 16x8 / 8x16 macroblock: neighbours A, B, C
// of the partition (C replaced by D when unavailable; blocks of the right neighbour are never
// available yet), the directional rules, else the median.  mv0: this MB's partition 0 vector.
MXHD Mv predict_mv_part(const MbNbrs& nb, const Avail& av, int part, int idx, Mv mv0) {
    MvNb own;
    own.avail = true;
    own.ref = 0;
    own.mv = mv0;
    MvNb a, b, c;
    if (part == kPart16x8) {
        if (idx == 0) {
            a = mv_nb_blk(nb.left, av.left, 3, 0);
            b = mv_nb_blk(nb.top, av.top, 0, 3);
            c = av.topright ? mv_nb_blk(nb.topright, true, 0, 3) : mv_nb_blk(nb.topleft, av.topleft, 3, 3);
            if (b.ref == 0) return b.mv;
        } else {
            a = mv_nb_blk(nb.left, av.left, 3, 2);
            b = own;
            c = mv_nb_blk(nb.left, av.left, 3, 1);  // C = (16, 7) not yet decoded -> D = (-1, 7)
            if (a.ref == 0) return a.mv;
        }
    } else {
        if (idx == 0) {
            a = mv_nb_blk(nb.left, av.left, 3, 0);
            b = mv_nb_blk(nb.top, av.top, 0, 3);
            c = av.top ? mv_nb_blk(nb.top, true, 2, 3) : mv_nb_blk(nb.topleft, av.topleft, 3, 3);
            if (a.ref == 0) return a.mv;
        } else {
            a = own;
            b = mv_nb_blk(nb.top, av.top, 2, 3);
            c = av.topright ? mv_nb_blk(nb.topright, true, 0, 3) : mv_nb_blk(nb.top, av.top, 1, 3);
            if (c.ref == 0) return c.mv;
        }
    }
    return predict_mv16x16(a, b, c);
}

// P_Skip decision + the motion vector differences of a P macroblock: mvd[0..1] (16x16 or
// partition 0), mvd[2..3] (partition 1).  Returns true for P_Skip (16x16 only).
MXHD bool decide_skip(const MbNbrs& nb, const Avail& av, int* mvd) {
    const MbInfo& m = *nb.self;
    mvd[0] = mvd[1] = mvd[2] = mvd[3] = 0;
    if (m.type != kMbP16x16) return false;
    if (m.part != kPart16x16) {
        const Mv v0{m.pmv[0], m.pmv[1]}, v1{m.pmv[2], m.pmv[3]};
        const Mv p0 = predict_mv_part(nb, av, m.part, 0, v0);
        const Mv p1 = predict_mv_part(nb, av, m.part, 1, v0);
        mvd[0] = v0.x - p0.x;
        mvd[1] = v0.y - p0.y;
        mvd[2] = v1.x - p1.x;
        mvd[3] = v1.y - p1.y;
        return false;
    }
    const MvNb a = mv_nb_blk(nb.left, av.left, 3, 0);
    const MvNb b = mv_nb_blk(nb.top, av.top, 0, 3);
    MvNb c = mv_nb_blk(nb.topright, av.topright, 0, 3);
    if (!av.topright) c = mv_nb_blk(nb.topleft, av.topleft, 3, 3);
    const Mv pskip = predict_mv_skip(a, b, c);
    const Mv p = predict_mv16x16(a, b, c);
    mvd[0] = m.mvx - p.x;
    mvd[1] = m.mvy - p.y;
    return m.cbp == 0 && m.mvx == pskip.x && m.mvy == pskip.y;
}

template <class W>
MXHD void code_role(W& w, int role, const Geometry& g, int idr, const MbNbrs& nb, const int16_t* mc,
                    const Avail& av, const int* mvd, int dqp = 0) {
    const MbInfo& m = *nb.self;
    const bool intra = m.type == kMbI16x16;  // Intra16x16: DC / AC split of the luma residual
    const int cbp = m.cbp;
    const int cbp_l = cbp & 15, cbp_c = cbp >> 4;
    const MbInfo* ml = av.left ? nb.left : nullptr;
    const MbInfo* mt = av.top ? nb.top : nullptr;
    if (role == 0) {
        if (intra) {
            const int mbtype = 1 + m.i16_mode + 4 * cbp_c + (cbp_l ? 12 : 0);
            put_ue(w, (uint32_t)(idr ? mbtype : 5 + mbtype));
            put_ue(w, m.chroma_mode);
            put_se(w, dqp);  // mb_qp_delta (0 in I slices: every MB at the slice QP)
        } else if (m.type == kMbI4x4) {
            put_ue(w, idr ? 0u : 5u);  // I_NxN
            // prev_intra4x4_pred_mode_flag / rem_intra4x4_pred_mode, blkIdx order (8.3.1.1:
            // a neighbour MB that is not Intra4x4 counts as DC, an unavailable one forces DC)
            for (int b = 0; b < 16; ++b) {
                const int bx = kBlkX[b], by = kBlkY[b];
                const bool ha = bx > 0 || av.left, hb = by > 0 || av.top;
                int ma = -1, mb = -1;
                if (bx > 0) ma = i4_get(m.i4, by * 4 + bx - 1);
                else if (ml && ml->type == kMbI4x4) ma = i4_get(ml->i4, by * 4 + 3);
                if (by > 0) mb = i4_get(m.i4, (by - 1) * 4 + bx);
                else if (mt && mt->type == kMbI4x4) mb = i4_get(mt->i4, 12 + bx);
                const int pm = i4_pred_mode(ma, mb, ha, hb);
                const int mode = i4_get(m.i4, by * 4 + bx);
                if (mode == pm) {
                    w.put(1, 1);
                } else {
                    w.put(0, 1);
                    w.put((uint32_t)(mode < pm ? mode : mode - 1), 3);
                }
            }
            put_ue(w, m.chroma_mode);
            put_ue(w, (uint32_t)cbp_to_codenum(cbp, true));
            if (cbp) put_se(w, dqp);
        } else {
            put_ue(w, m.part);  // P_L0_16x16 / P_L0_L0_16x8 / P_L0_L0_8x16 (one reference: no ref_idx)
            put_se(w, mvd[0]);
            put_se(w, mvd[1]);
            if (m.part != kPart16x16) {
                put_se(w, mvd[2]);
                put_se(w, mvd[3]);
            }
            put_ue(w, (uint32_t)cbp_to_codenum(cbp, false));
            if (cbp) put_se(w, dqp);  // mb_qp_delta (adaptive quantisation)
        }
        return;
    }
    if (role == 1) {
        if (!intra) return;
        const int nc = combine_nc(av.left, ml ? ml->nz_luma[3] : 0, av.top, mt ? mt->nz_luma[12] : 0);
        cavlc_block(w, mc + kCoefLumaDc, 16, nc);
        return;
    }
    if (role <= 17) {
        const int b = role - 2;
        if (!(cbp_l & (1 << (b >> 2)))) return;
        const int bx = kBlkX[b], by = kBlkY[b];
        const bool ha = bx > 0 || av.left, hb = by > 0 || av.top;
        const int na = bx > 0 ? m.nz_luma[by * 4 + bx - 1] : (ml ? ml->nz_luma[by * 4 + 3] : 0);
        const int nb = by > 0 ? m.nz_luma[(by - 1) * 4 + bx] : (mt ? mt->nz_luma[12 + bx] : 0);
        const int nc = combine_nc(ha, na, hb, nb);
        if (intra) {
            cavlc_block(w, mc + kCoefLuma + b * 16 + 1, 15, nc);  // AC only (DC in the Intra16x16 DC block)
        } else {
            cavlc_block(w, mc + kCoefLuma + b * 16, 16, nc);
        }
        return;
    }
    if (role <= 19) {
        if (!cbp_c) return;
        const int comp = role - 18;
        cavlc_block(w, mc + kCoefChromaDc + comp * 4, 4, -1);
        return;
    }
    if (role < kNumRoles) {
        if (cbp_c != 2) return;
        const int comp = (role - 20) >> 2, cb = (role - 20) & 3, bx = cb & 1, by = cb >> 1;
        const uint8_t* own = comp ? m.nz_cr : m.nz_cb;
        const uint8_t* lft = ml ? (comp ? ml->nz_cr : ml->nz_cb) : nullptr;
        const uint8_t* top = mt ? (comp ? mt->nz_cr : mt->nz_cb) : nullptr;
        const bool ha = bx > 0 || av.left, hb = by > 0 || av.top;
        const int na = bx > 0 ? own[by * 2] : (lft ? lft[by * 2 + 1] : 0);
        const int nb = by > 0 ? own[bx] : (top ? top[2 + bx] : 0);
        const int nc = combine_nc(ha, na, hb, nb);
        cavlc_block(w, mc + kCoefChromaAc + (comp * 4 + cb) * 16 + 1, 15, nc);
    }
}

// Adaptive quantisation (residual-energy based, P macroblocks): a block whose motion-
// compensated luma residual stays noise-like (mean |residual| above 32 / 48 per pixel) is
// quantised 6 / 12 QP coarser -- refining incompressible content costs far more bits than
// it returns -- and the rate controller hands those bits to the rest of the picture (text,
// UI edges).  sad = sum |src - pred| over the 16x16 luma block.
MXHD int aq_mb_qp(int frame_qp, uint32_t sad, int aq) {
    if (!aq) return frame_qp;  // (aq 3 -- the temporal classes below -- falls back to this rule in HEVC)
    const int off = sad > 256u * 48 ? 12 : (sad > 256u * 32 ? 6 : 0);
    const int q = frame_qp + off;
    return q > 51 ? 51 : q;
}

// Rate-distortion residual drop for noise-like P macroblocks (EncoderConfig::aq >= 2).  A
// macroblock in an AQ noise class (mean |luma residual| above 32 per pixel) keeps its residual
// only if coding it lowers the luma distortion by more than lambda * (estimated bits):
// refining incompressible content at the QPs a CBR budget allows costs far more than it
// returns, and the rate controller hands those bits to the rest of the picture.  lambda is
// the H.264 reference mode-decision lambda 0.85 * 2^((qp - 12) / 3) (SSE domain), the bit
// estimate 2 + 6 per non-zero coefficient per 4x4 block.
MXHD int lambda_sse(int qp) {
    constexpr int tab[52] = {0,   0,   0,   0,   0,   0,   0,   0,   0,    0,    1,    1,    1,    1,
                             1,   2,   2,   3,   3,   4,   5,   7,   9,    11,   14,   17,   22,   27,
                             34,  43,  54,  69,  86,  109, 137, 173, 218,  274,  345,  435,  548,  691,
                             870, 1097, 1382, 1741, 2193, 2763, 3482, 4387, 5527, 6963};
    return tab[qp < 0 ? 0 : (qp > 51 ? 51 : qp)];
}
MXHD uint32_t block_bits_est(int nz) { return nz ? 2u + 6u * (uint32_t)nz : 0u; }
MXHD bool drop_residual(int aq, uint32_t lsad, int qp, long long d_pred, long long d_coded, uint32_t bits) {
    if (aq < 2 || lsad <= 256u * 32) return false;
    return d_pred - d_coded < (long long)lambda_sse(qp) * (long long)bits;
}

// Temporal classes (EncoderConfig::aq == 3, the H.264 default).  The residual-energy rule above
// cannot tell incompressible content from well-predictable content whose reference is still
// coarse: text coded at a high QP in the IDR leaves a large residual too, and was then quantised
// 6-12 QP coarser -- never refined (the document window stayed at 28 dB over the driver window,
// tools/region_report.py).  The classes here use the SOURCE's own temporal change instead:
// tsad = sum |src_n - src_(n-1)| over the 16x16 luma block displaced by the integer part of the
// chosen motion vector.
//  * changing content (tsad > 24 / pixel: e.g. animated noise, video): its bits are thrown away
//    with the next picture -> 6 QP coarser, luma residual kept only if it pays for its bits
//    (drop_residual's rate-distortion rule), chroma residual dropped;
//  * persistent content (tsad <= 2 / pixel: static or moving rigidly): everything coded now is
//    re-used by every later picture (the static desktop refines once and is then skipped) ->
//    6 QP finer -- a one-step form of x264's macroblock-tree propagation without a lookahead;
//  * anything else at the frame QP.
constexpr uint32_t kTsadChanging = 256u * 24, kTsadPersistent = 256u * 2;
constexpr int kAqChangingOffset = 6, kAqPersistentOffset = -6;
// Static content (aq >= 4): a block whose source is bit-identical to the previous source with a zero
// vector is coded once and then skipped for as long as it stays -- refined 9 / 12 / 15 QP finer
// (aq 4 / 5 / 6) than the frame QP; only rigidly MOVING persistent content (a pan, a scroll) keeps
// -6, since there every frame re-spends the finer QP on the newly exposed / re-predicted blocks and
// the rate control raises the frame QP for everything (profiles/r04_hevc/NOTES.md: aq 5 on the
// motion content cost 5 dB when the offset applied to every persistent block).
MXHD int aq_static_offset(int aq) { return kAqPersistentOffset - 3 * ((aq > 6 ? 6 : aq) - 3); }
enum TClass : int { kTcNormal = 0, kTcPersistent = 1, kTcChanging = 2, kTcStatic = 3 };
MXHD int temporal_class(uint32_t tsad, bool zero_mv) {
    return tsad > kTsadChanging ? kTcChanging
                                : (tsad == 0 && zero_mv ? kTcStatic : (tsad <= kTsadPersistent ? kTcPersistent : kTcNormal));
}
MXHD int aq3_mb_qp(int frame_qp, int tclass, int aq = 3) {
    const int q = frame_qp + (tclass == kTcChanging     ? kAqChangingOffset
                              : tclass == kTcStatic     ? aq_static_offset(aq)
                              : tclass == kTcPersistent ? kAqPersistentOffset
                                                        : 0);
    return q < 0 ? 0 : (q > 51 ? 51 : q);
}
// MB QP and residual-drop decision of a P macroblock for any aq mode (aq >= 3 uses tclass).
MXHD int mb_qp_for(int frame_qp, uint32_t lsad, int tclass, int aq) {
    return aq >= 3 ? aq3_mb_qp(frame_qp, tclass, aq) : aq_mb_qp(frame_qp, lsad, aq);
}
MXHD bool drop_luma_for(int aq, uint32_t lsad, int tclass, int qp, long long d_pred, long long d_coded,
                        uint32_t bits) {
    if (aq >= 3)
        return tclass == kTcChanging && d_pred - d_coded < (long long)lambda_sse(qp) * (long long)bits;
    return drop_residual(aq, lsad, qp, d_pred, d_coded, bits);
}
MXHD bool drop_chroma_for(int aq, int tclass, bool luma_dropped) {
    return luma_dropped || (aq >= 3 && tclass == kTcChanging);
}

// Inter cost of a P16x16 macroblock for the intra decision: luma SATD of the motion-
// compensated residual + mv rate at the frame lambda.
MXHD uint32_t inter_cost(uint32_t satd, int frame_qp, int mvx, int mvy) {
    return satd + (uint32_t)(lambda_sad(frame_qp) * (mvd_bits(mvx) + mvd_bits(mvy)));
}
// ... of a partitioned macroblock: both vectors' rate
MXHD uint32_t inter_cost_mb(uint32_t satd, int frame_qp, const MbInfo& m) {
    if (m.part == kPart16x16) return inter_cost(satd, frame_qp, m.mvx, m.mvy);
    return satd + (uint32_t)(lambda_sad(frame_qp) *
                             (mvd_bits(m.pmv[0]) + mvd_bits(m.pmv[1]) + mvd_bits(m.pmv[2]) + mvd_bits(m.pmv[3])));
}

// Rows per slice of an IDR picture: intra macroblocks are reconstructed in a diagonal
// wavefront per slice (one workgroup per slice, one wave per row, k_intra_wave), so a slice
// takes about as long as its most expensive MB row plus a 2-MB lag per row.  <= 4-row slices
// (17 at 1080p) keep one row wave per SIMD and spread the text-heavy rows over more
// workgroups: 1,059 -> 914 us per 1080p IDR against 8-row slices for +0.7 % IDR bytes
// (profiles/r02_idr).
MXHD int idr_slice_rows(int mb_h) {
    const int ns = (mb_h + 3) / 4;  // <= 4 rows
    return (mb_h + ns - 1) / ns;
}

// mb_qp_delta value for QP `qp` after predictor `pred` (both 0..51), in -26..25.
MXHD int qp_delta(int qp, int pred) { return ((qp - pred + 26 + 52) % 52) - 26; }

MXHD SliceParams make_slice_params(int first_mb, int idr, int frame_num, int log2_max_frame_num, int idr_pic_id,
                                   int qp_delta, int deblock_off) {
    SliceParams sp;
    sp.first_mb = first_mb;
    sp.idr = idr;
    sp.frame_num = frame_num;
    sp.log2_max_frame_num = log2_max_frame_num;
    sp.idr_pic_id = idr_pic_id;
    sp.qp_delta = qp_delta;
    sp.disable_deblock = deblock_off;
    return sp;
}

// ---- per-block transform pipelines (same arithmetic on both encoders)

// Inter luma block: residual (raster) -> levels (scan order) + reconstructed residual.
MXHD int luma_block_inter(const int* res, int qp, int* zscan, int* rres) {
    int y[16], z[16], d[16];
    fdct4x4(res, y);
    const int nz = quant4x4(y, z, qp, false, 0);
    for (int k = 0; k < 16; ++k) zscan[k] = z[kZigzag4x4[k]];
    dequant4x4(z, d, qp, 0);
    idct4x4(d, rres);
    return nz;
}

// ME cost shared by both encoders.
MXHD uint32_t me_cost(uint32_t sad, int lambda, int mvx, int mvy) {
    return sad + (uint32_t)(lambda * (mvd_bits(mvx) + mvd_bits(mvy)));
}

// Integer search radius actually used: clamped to [4, 32] and rounded up to a multiple of
// 4 so the search window starts on a dword boundary.
MXHD int me_range(int r) {
    r = r < 4 ? 4 : (r > 32 ? 32 : r);
    return (r + 3) & ~3;
}
// Static-block early exit: a zero vector with SAD <= static_sad(qp) ends the search (both
// encoders apply the same rule, so their decisions stay bit-identical).  The reference is the
// lossy reconstruction, so an unchanged desktop region differs from it by the coding noise of
// the previous picture; a fixed threshold (128 = 0.5 per pixel) sent nearly every static MB of
// a QP-36 desktop through the full search (profiles/r02_c: ~1100 VALU per wave in k_me_full).
// A flat 16x16 residual of r per sample quantises to zero while r < ~qstep/4.7 (inter dead
// zone, 4x4 DC); 64 * lambda_sad(qp) ~ 256 * qstep / 12 stays well inside that.
constexpr uint32_t kStaticSad = 128;
MXHD uint32_t static_sad(int qp) {
    const uint32_t t = 64u * (uint32_t)lambda_sad(qp);
    return t > kStaticSad ? t : kStaticSad;
}

// Sub-pel refinement neighbour k (0..7) offsets.
MXHD void subpel_offset(int k, int* dx, int* dy) {
    *dx = (k < 3) ? (k - 1) : (k == 3 ? -1 : (k == 4 ? 1 : (k - 6)));
    *dy = (k < 3) ? -1 : ((k == 3 || k == 4) ? 0 : 1);
}

}  // namespace h264
}  // namespace mx
