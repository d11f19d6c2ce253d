// VP8 frame writer (RFC 6386 sections 9, 13, 16, 17, 19): frame tag, key-frame start code and
// size, the first partition (frame header + per-macroblock modes and motion vectors) and the
// token partitions (one per MB row modulo the partition count, written concurrently -- a token
// partition's contexts depend only on the coefficients, which are known before coding starts).
#include <exception>
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "vp8_encoder.h"

namespace mx {
namespace vp8 {

namespace {

inline int coef_index(int type, int band, int ctx) { return ((type * 8 + band) * 3 + ctx) * 11; }

// Token coding over a probability table: Enc::tok(table index, bit) codes (or counts) a
// context-coded token branch, Enc::fix(prob, bit) a fixed-probability bit (extra bits, sign).
struct TokWriter {
    BoolEncoder& e;
    const uint8_t* probs;
    void tok(int idx, int bit) { e.put(probs[idx], bit); }
    void fix(int prob, int bit) { e.put(prob, bit); }
};
struct TokWriterCount {  // coding + branch statistics for the next frame's probability updates (13.4)
    BoolEncoder& e;
    const uint8_t* probs;
    uint32_t (*n)[2];
    void tok(int idx, int bit) {
        e.put(probs[idx], bit);
        ++n[idx][bit];
    }
    void fix(int prob, int bit) { e.put(prob, bit); }
};

template <class Enc>
void put_extra(Enc& e, int v, const uint8_t* p, int n) {
    for (int k = n - 1; k >= 0; --k) e.fix(p[n - 1 - k], (v >> k) & 1);
}

// One block's tokens (13.2 / 13.3).
template <class Enc>
void put_block(Enc& e, const int16_t* lv, int first, int type, int ctx) {
    int last = 15;
    while (last >= first && lv[last] == 0) --last;
    if (last < first) {
        e.tok(coef_index(type, kBand[first], ctx) + 0, 0);  // EOB
        return;
    }
    bool prev_zero = false;
    for (int i = first; i <= last; ++i) {
        const int P = coef_index(type, kBand[i], ctx);
        if (!prev_zero) e.tok(P + 0, 1);  // not EOB
        const int v = lv[i], a = v < 0 ? -v : v;
        if (a == 0) {
            e.tok(P + 1, 0);
            ctx = 0;
            prev_zero = true;
            continue;
        }
        e.tok(P + 1, 1);
        if (a == 1) {
            e.tok(P + 2, 0);
        } else {
            e.tok(P + 2, 1);
            if (a <= 4) {
                e.tok(P + 3, 0);
                if (a == 2) {
                    e.tok(P + 4, 0);
                } else {
                    e.tok(P + 4, 1);
                    e.tok(P + 5, a == 4);
                }
            } else {
                e.tok(P + 3, 1);
                if (a <= 10) {
                    e.tok(P + 6, 0);
                    if (a <= 6) {
                        e.tok(P + 7, 0);
                        put_extra(e, a - 5, kPcat1, 1);
                    } else {
                        e.tok(P + 7, 1);
                        put_extra(e, a - 7, kPcat2, 2);
                    }
                } else {
                    e.tok(P + 6, 1);
                    if (a <= 34) {
                        e.tok(P + 8, 0);
                        if (a <= 18) {
                            e.tok(P + 9, 0);
                            put_extra(e, a - 11, kPcat3, 3);
                        } else {
                            e.tok(P + 9, 1);
                            put_extra(e, a - 19, kPcat4, 4);
                        }
                    } else {
                        e.tok(P + 8, 1);
                        if (a <= 66) {
                            e.tok(P + 10, 0);
                            put_extra(e, a - 35, kPcat5, 5);
                        } else {
                            e.tok(P + 10, 1);
                            put_extra(e, a - 67, kPcat6, 11);
                        }
                    }
                }
            }
        }
        e.fix(128, v < 0);
        ctx = a == 1 ? 1 : 2;
        prev_zero = false;
    }
    if (last < 15) e.tok(coef_index(type, kBand[last + 1], ctx) + 0, 0);  // EOB
}

inline int nzb(const Vp8Mb& m, int b) { return (m.nz >> b) & 1; }

// A sub-block mode through the bmode tree (11.2; bmode_cost256 walks the same branches).
template <class Enc>
void put_bmode(Enc& e, int m, const uint8_t* p) {
    e.put(p[0], m != kBDc);
    if (m == kBDc) return;
    e.put(p[1], m != kBTm);
    if (m == kBTm) return;
    e.put(p[2], m != kBVe);
    if (m == kBVe) return;
    const bool far = !(m == kBHe || m == kBRd || m == kBVr);
    e.put(p[3], far);
    if (!far) {
        e.put(p[4], m != kBHe);
        if (m != kBHe) e.put(p[5], m == kBVr);
        return;
    }
    e.put(p[6], m != kBLd);
    if (m == kBLd) return;
    e.put(p[7], m != kBVl);
    if (m != kBVl) e.put(p[8], m == kBHu);
}

// Y2 "above" context of macroblock (mbx, mby): the Y2 block's non-zero bit of the nearest macroblock
// above with a Y2 block -- B_PRED macroblocks have none and leave the column's context as it was
// (a skipped 16x16 macroblock resets it: its nz bits are 0)
inline int y2_above(const Vp8Mb* mbs, int mb_w, int mbx, int mby) {
    for (int y = mby - 1; y >= 0; --y) {
        const Vp8Mb& u = mbs[y * mb_w + mbx];
        if (u.ymode != kBPred) return nzb(u, kY2);
    }
    return 0;
}

// Token partition `p`: MB rows p, p + n, ...
template <class Enc>
void code_tokens(const FrameDesc& f, const Vp8Mb* mbs, const std::function<const int16_t*(int)>& levels, int p, int n,
                 Enc& e) {
    for (int mby = p; mby < f.mb_h; mby += n) {
        int left[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // Y0..3 (rows), U0..1, V0..1, Y2
        for (int mbx = 0; mbx < f.mb_w; ++mbx) {
            const int i = mby * f.mb_w + mbx;
            const Vp8Mb& m = mbs[i];
            const bool y2 = m.ymode != kBPred;
            if (m.nz == 0) {  // mb_skip_coeff: no tokens, contexts reset (Y2's only with a Y2 block)
                for (int k = 0; k < 8; ++k) left[k] = 0;
                if (y2) left[8] = 0;
                continue;
            }
            const Vp8Mb* up = mby > 0 ? &mbs[i - f.mb_w] : nullptr;
            const int16_t* lv = levels(i);
            if (y2) {  // Y2 (type 1)
                const int ctx = y2_above(mbs, f.mb_w, mbx, mby) + left[8];
                put_block(e, lv + kY2 * 16, 0, 1, ctx);
                left[8] = nzb(m, kY2);
            }
            for (int b = 0; b < 16; ++b) {  // Y: after Y2 type 0 from coefficient 1; B_PRED type 3 from 0
                const int bx = b & 3, by = b >> 2;
                const int above = by > 0 ? nzb(m, b - 4) : (up ? nzb(*up, 12 + bx) : 0);
                put_block(e, lv + b * 16, y2 ? 1 : 0, y2 ? 0 : 3, above + left[by]);
                left[by] = nzb(m, b);
            }
            for (int c = 0; c < 2; ++c)
                for (int b = 0; b < 4; ++b) {  // chroma (type 2)
                    const int blk = 16 + 4 * c + b, bx = b & 1, by = b >> 1;
                    const int above = by > 0 ? nzb(m, blk - 2) : (up ? nzb(*up, blk + 2) : 0);
                    put_block(e, lv + blk * 16, 0, 2, above + left[4 + 2 * c + by]);
                    left[4 + 2 * c + by] = nzb(m, blk);
                }
        }
    }
}

// Cost in 1/256 bit of coding `bit` at probability `prob` (of a zero): -256 log2(p).
inline int bit_cost256(int prob, int bit) {
    static const auto tab = [] {
        std::array<int, 256> t{};
        for (int k = 1; k < 256; ++k) t[k] = (int)std::lround(-256.0 * std::log2(k / 256.0));
        t[0] = t[1];
        return t;
    }();
    return tab[bit ? 256 - prob : prob];
}

// Per-frame coefficient probability updates (13.4): a probability is replaced by its frame's
// optimum when the branch statistics save more than the update costs (the flag at its update
// probability + 8 bits).  refresh_entropy_probs stays 0, so every frame updates against the
// defaults.  upd[k] = the new probability or 0.
void plan_prob_updates(const uint32_t (*n)[2], uint8_t* upd, uint8_t* probs) {
    for (int k = 0; k < 1056; ++k) {
        upd[k] = 0;
        probs[k] = kCoefProbs0[k];
        const uint32_t n0 = n[k][0], n1 = n[k][1], t = n0 + n1;
        if (t == 0) continue;
        const int np = std::clamp((int)((n0 * 256ull + t / 2) / t), 1, 255);
        if (np == kCoefProbs0[k]) continue;
        const long long old_c = (long long)n0 * bit_cost256(kCoefProbs0[k], 0) + (long long)n1 * bit_cost256(kCoefProbs0[k], 1);
        const long long new_c = (long long)n0 * bit_cost256(np, 0) + (long long)n1 * bit_cost256(np, 1);
        const long long flag = bit_cost256(kCoefUpdateProbs[k], 1) - bit_cost256(kCoefUpdateProbs[k], 0);
        if (old_c - new_c > flag + 8 * 256) {
            upd[k] = (uint8_t)np;
            probs[k] = (uint8_t)np;
        }
    }
}

inline void clamp_mv(int mv[2], int mb_w, int mb_h, int mbx, int mby) {
    // vp8_clamp_mv2: the block may reach 16 samples beyond the picture (1/8-sample units)
    const int lo_x = -((mbx * 16) << 3) - (16 << 3), hi_x = (((mb_w - 1 - mbx) * 16) << 3) + (16 << 3);
    const int lo_y = -((mby * 16) << 3) - (16 << 3), hi_y = (((mb_h - 1 - mby) * 16) << 3) + (16 << 3);
    mv[0] = std::clamp(mv[0], lo_x, hi_x);
    mv[1] = std::clamp(mv[1], lo_y, hi_y);
}

void put_mv_component(BoolEncoder& e, int v, const uint8_t* p) {
    // v in quarter samples (the decoder doubles it)
    const int a = v < 0 ? -v : v;
    if (a < 8) {
        e.put(p[0], 0);
        // small tree: {2, 8, 4, 6, -0, -1, -2, -3, 10, 12, -4, -5, -6, -7}, probabilities p[2 + node / 2]
        e.put(p[2], a >= 4);
        if (a < 4) {
            e.put(p[3], a >= 2);
            e.put(p[a < 2 ? 4 : 5], a & 1);
        } else {
            e.put(p[6], a >= 6);
            e.put(p[a < 6 ? 7 : 8], a & 1);
        }
        if (a) e.put(p[1], v < 0);
        return;
    }
    e.put(p[0], 1);
    for (int i = 0; i < 3; ++i) e.put(p[9 + i], (a >> i) & 1);
    for (int i = 9; i > 3; --i) e.put(p[9 + i], (a >> i) & 1);
    if (a & 0xfff0) e.put(p[9 + 3], (a >> 3) & 1);
    e.put(p[1], v < 0);
}

}  // namespace

void find_near_mvs(const Vp8Mb* mbs, int mb_w, int mb_h, int mbx, int mby, int near_mv[3][2], int cnt[4]) {
    int mv[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
    int idx = 0;  // index of the last distinct vector stored
    auto is_inter = [&](int x, int y) { return x >= 0 && y >= 0 && x < mb_w && mbs[y * mb_w + x].ymode == kInter; };
    auto mv_of = [&](int x, int y, int o[2]) {
        o[0] = mbs[y * mb_w + x].mvx;
        o[1] = mbs[y * mb_w + x].mvy;
    };
    // above (weight 2), left (2), above-left (1); outside the picture counts as intra
    const int nx[3] = {mbx, mbx - 1, mbx - 1}, ny[3] = {mby - 1, mby, mby - 1}, wt[3] = {2, 2, 1};
    for (int k = 0; k < 3; ++k) {
        if (!is_inter(nx[k], ny[k])) continue;
        int t[2];
        mv_of(nx[k], ny[k], t);
        if (t[0] | t[1]) {
            if (k == 0 || t[0] != mv[idx][0] || t[1] != mv[idx][1]) {
                ++idx;
                mv[idx][0] = t[0];
                mv[idx][1] = t[1];
            }
            cnt[idx] += wt[k];
        } else {
            cnt[0] += wt[k];
        }
    }
    // three distinct vectors and the last equals the first: the nearest gains a vote
    if (cnt[3] && mv[idx][0] == mv[1][0] && mv[idx][1] == mv[1][1]) cnt[1] += 1;
    cnt[3] = 0;  // no SPLITMV neighbours
    if (cnt[2] > cnt[1]) {
        std::swap(cnt[1], cnt[2]);
        std::swap(mv[1][0], mv[2][0]);
        std::swap(mv[1][1], mv[2][1]);
    }
    if (cnt[1] >= cnt[0]) {
        mv[0][0] = mv[1][0];
        mv[0][1] = mv[1][1];
    }
    for (int k = 0; k < 3; ++k) {
        near_mv[k][0] = mv[k][0];
        near_mv[k][1] = mv[k][1];
        clamp_mv(near_mv[k], mb_w, mb_h, mbx, mby);
    }
}

void write_frame(const FrameDesc& f, const Vp8Mb* mbs, const std::function<const int16_t*(int)>& levels,
                 std::vector<uint8_t>& out,
                 const std::function<void(int, const std::function<void(int)>&)>& run_parallel, TokenStats* stats) {
    const int nmb = f.mb_w * f.mb_h;
    const int nparts = 1 << f.log2_parts;
    int coded = 0, intra = 0;
    for (int i = 0; i < nmb; ++i) {
        coded += mbs[i].nz != 0;
        intra += mbs[i].ymode != kInter;
    }
    const int prob_skip_false = std::clamp((coded * 256 + nmb / 2) / std::max(1, nmb), 1, 255);
    // inter frames: the probability of an intra macroblock (intra_pass), from this frame's count
    const int prob_intra = std::clamp((intra * 256 + nmb / 2) / std::max(1, nmb), 1, 255);
    // segment tree probabilities (9.3, mb_segment_tree {2, 4, -0, -1, -2, -3}) from this frame's
    // segment histogram: p0 = P(segment < 2), p1 = P(1 | < 2), p2 = P(3 | >= 2)
    int seg_n[kNumSegs] = {0, 0, 0, 0};
    if (f.segmented)
        for (int i = 0; i < nmb; ++i) ++seg_n[mbs[i].seg & 3];
    auto prob_of = [](int zero, int total) { return total ? std::clamp((zero * 256 + total / 2) / total, 1, 255) : 255; };
    const int seg_p[3] = {prob_of(seg_n[0] + seg_n[1], nmb), prob_of(seg_n[0], seg_n[0] + seg_n[1]),
                          prob_of(seg_n[2], seg_n[2] + seg_n[3])};
    // ---- probability updates planned from the previous frame's branch statistics of this type
    uint8_t upd[1056], probs[1056];
    if (stats && stats->valid) {
        plan_prob_updates(reinterpret_cast<const uint32_t(*)[2]>(stats->n[0].data()), upd, probs);
    } else {
        std::memset(upd, 0, sizeof upd);
        std::memcpy(probs, kCoefProbs0, sizeof probs);
    }
    // ---- first partition (a job beside the token partitions: it reads only modes / vectors)
    std::vector<uint8_t> p1;
    p1.reserve(16 + (size_t)nmb / 2);
    auto code_first = [&]() {
        BoolEncoder e(p1);
        if (f.key) {
            e.literal(0, 1);  // color_space
            e.literal(0, 1);  // clamping_type (decoder clamps reconstructed samples)
        }
        e.literal(f.segmented ? 1 : 0, 1);  // segmentation_enabled
        if (f.segmented) {
            e.literal(1, 1);  // update_mb_segmentation_map
            e.literal(1, 1);  // update_segment_feature_data
            e.literal(1, 1);  // segment_feature_mode: absolute values
            for (int k = 0; k < kNumSegs; ++k) {  // quantizer: the segment's y_ac_qi
                e.literal(1, 1);
                e.literal((uint32_t)f.seg_qindex[k], 7);
                e.literal(0, 1);  // sign
            }
            for (int k = 0; k < kNumSegs; ++k) {  // loop-filter level: the segment's (absolute)
                e.literal(f.lf_level[k] != 0, 1);
                if (f.lf_level[k]) {
                    e.literal((uint32_t)f.lf_level[k], 6);
                    e.literal(0, 1);  // sign
                }
            }
            for (int k = 0; k < 3; ++k) {  // segment tree probabilities
                e.literal(1, 1);
                e.literal((uint32_t)seg_p[k], 8);
            }
        }
        // the frame level only switches the filter on (segmented frames: each segment's own level)
        int frame_level = f.lf_level[0];
        if (f.segmented)
            for (int k = 1; k < kNumSegs; ++k) frame_level = std::max(frame_level, f.lf_level[k]);
        e.literal(0, 1);  // filter_type (normal)
        e.literal((uint32_t)frame_level, 6);  // loop_filter_level (0: no loop filter)
        e.literal(0, 3);  // sharpness_level
        e.literal(0, 1);  // loop_filter_adj_enable
        e.literal((uint32_t)f.log2_parts, 2);
        e.literal((uint32_t)f.qindex, 7);  // y_ac_qi
        for (int k = 0; k < 5; ++k) e.literal(0, 1);  // no quantiser deltas
        if (f.key) {
            e.literal(0, 1);  // refresh_entropy_probs: probabilities of this frame not kept
        } else {
            e.literal(0, 1);  // refresh_golden_frame
            e.literal(0, 1);  // refresh_alternate_frame
            e.literal(0, 2);  // copy_buffer_to_golden: none
            e.literal(0, 2);  // copy_buffer_to_alternate: none
            e.literal(0, 1);  // sign_bias_golden
            e.literal(0, 1);  // sign_bias_alternate
            e.literal(0, 1);  // refresh_entropy_probs
            e.literal(1, 1);  // refresh_last
        }
        for (int k = 0; k < 1056; ++k) {  // token probability updates (plan_prob_updates)
            e.put(kCoefUpdateProbs[k], upd[k] != 0);
            if (upd[k]) e.literal(upd[k], 8);
        }
        e.literal(1, 1);  // mb_no_skip_coeff
        e.literal((uint32_t)prob_skip_false, 8);
        const int prob_last = 255, prob_gf = 128;
        if (!f.key) {
            e.literal(prob_intra, 8);
            e.literal(prob_last, 8);
            e.literal(prob_gf, 8);
            e.literal(0, 1);  // intra_16x16_prob_update_flag
            e.literal(0, 1);  // intra_chroma_prob_update_flag
            for (int c = 0; c < 2; ++c)
                for (int k = 0; k < 19; ++k) e.put(kMvUpdateProbs[c][k], 0);  // no mv probability updates
        }
        for (int mby = 0; mby < f.mb_h; ++mby)
            for (int mbx = 0; mbx < f.mb_w; ++mbx) {
                const Vp8Mb& m = mbs[mby * f.mb_w + mbx];
                if (f.segmented) {  // segment_id
                    const int sg = m.seg & 3;
                    e.put(seg_p[0], sg >= 2);
                    e.put(sg >= 2 ? seg_p[2] : seg_p[1], sg & 1);
                }
                e.put(prob_skip_false, m.nz == 0);
                if (f.key) {
                    const uint8_t* p = kKfYModeProb;  // tree: B_PRED "0", DC "100", V "101", H "110", TM "111"
                    e.put(p[0], m.ymode != kBPred);
                    if (m.ymode == kBPred) {  // 16 sub-block modes under their above / left contexts
                        for (int b = 0; b < 16; ++b) {
                            const int bx = b & 3, by = b >> 2;
                            const int a = by > 0 ? bmode_of(m, b - 4) : bctx_above(mbs, f.mb_w, mbx, mby, bx);
                            const int l = bx > 0 ? bmode_of(m, b - 1) : bctx_left(mbs, f.mb_w, mbx, mby, by);
                            put_bmode(e, bmode_of(m, b), kKfBModeProb + (a * kNumBModes + l) * 9);
                        }
                    } else {
                        e.put(p[1], m.ymode >= kHPred);
                        e.put(m.ymode >= kHPred ? p[3] : p[2], m.ymode == kVPred || m.ymode == kTmPred);
                    }
                    const uint8_t* q = kKfUvModeProb;  // DC "0", V "10", H "110", TM "111"
                    e.put(q[0], m.uvmode != kDcPred);
                    if (m.uvmode != kDcPred) {
                        e.put(q[1], m.uvmode != kVPred);
                        if (m.uvmode != kVPred) e.put(q[2], m.uvmode == kTmPred);
                    }
                    continue;
                }
                if (m.ymode != kInter) {  // intra macroblock (16x16 modes): the inter-frame mode trees
                    if (m.ymode > kTmPred) throw std::logic_error("vp8 writer: B_PRED in an inter frame");
                    e.put(prob_intra, 0);     // is_inter_mb
                    const uint8_t* p = kYModeProb;  // DC "0", V "100", H "101", TM "110", B_PRED "111"
                    e.put(p[0], m.ymode != kDcPred);
                    if (m.ymode != kDcPred) {
                        e.put(p[1], m.ymode == kTmPred);
                        if (m.ymode == kTmPred)
                            e.put(p[3], 0);
                        else
                            e.put(p[2], m.ymode == kHPred);
                    }
                    const uint8_t* q = kUvModeProb;  // DC "0", V "10", H "110", TM "111"
                    e.put(q[0], m.uvmode != kDcPred);
                    if (m.uvmode != kDcPred) {
                        e.put(q[1], m.uvmode != kVPred);
                        if (m.uvmode != kVPred) e.put(q[2], m.uvmode == kTmPred);
                    }
                    continue;
                }
                e.put(prob_intra, 1);  // is_inter_mb
                e.put(prob_last, 0);   // reference: last frame
                if (m.mvx == 0 && m.mvy == 0) {
                    // ZEROMV needs only cnt[0] of find_near_mvs: the weights of the inter
                    // neighbours (above 2, left 2, above-left 1) with a zero vector
                    auto zero_at = [&](int x, int y) {
                        if (x < 0 || y < 0) return false;
                        const Vp8Mb& q = mbs[y * f.mb_w + x];
                        return q.ymode == kInter && q.mvx == 0 && q.mvy == 0;
                    };
                    const int c0 = 2 * zero_at(mbx, mby - 1) + 2 * zero_at(mbx - 1, mby) + zero_at(mbx - 1, mby - 1);
                    e.put(kModeContexts[c0][0], 0);
                    continue;
                }
                int near[3][2], cnt[4];
                find_near_mvs(mbs, f.mb_w, f.mb_h, mbx, mby, near, cnt);
                const uint8_t pr[4] = {kModeContexts[cnt[0]][0], kModeContexts[cnt[1]][1], kModeContexts[cnt[2]][2],
                                       kModeContexts[cnt[3]][3]};
                if (m.mvx == 0 && m.mvy == 0) {
                    e.put(pr[0], 0);  // ZEROMV
                    continue;
                }
                e.put(pr[0], 1);
                if (m.mvx == near[1][0] && m.mvy == near[1][1]) {
                    e.put(pr[1], 0);  // NEARESTMV
                    continue;
                }
                e.put(pr[1], 1);
                if (m.mvx == near[2][0] && m.mvy == near[2][1]) {
                    e.put(pr[2], 0);  // NEARMV
                    continue;
                }
                e.put(pr[2], 1);
                e.put(pr[3], 0);  // NEWMV (not SPLITMV)
                put_mv_component(e, (m.mvy - near[0][1]) / 2, kMvDefault[0]);  // row first
                put_mv_component(e, (m.mvx - near[0][0]) / 2, kMvDefault[1]);
            }
        e.flush();
    };
    // ---- token partitions, concurrently, over the updated probabilities (counting this frame's
    // branch statistics on the way when the caller keeps them)
    std::vector<std::vector<uint8_t>> parts((size_t)nparts);
    std::vector<std::array<uint32_t, 2>> cnt(stats ? (size_t)nparts * 1056 : 0, std::array<uint32_t, 2>{0u, 0u});
    std::exception_ptr first_err;
    std::vector<double> job_us((size_t)nparts + 1, 0.0);
    run_parallel(nparts + 1, [&](int j) {
        const auto t0 = std::chrono::steady_clock::now();
        struct Acc {
            double& a;
            std::chrono::steady_clock::time_point t;
            ~Acc() { a = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count(); }
        } acc{job_us[(size_t)j], t0};
        if (j == 0) {
            try {
                code_first();
            } catch (...) {
                first_err = std::current_exception();
            }
            return;
        }
        const int p = j - 1;
        parts[(size_t)p].reserve(4096);
        BoolEncoder e(parts[(size_t)p]);
        if (stats) {
            TokWriterCount w{e, probs, reinterpret_cast<uint32_t(*)[2]>(cnt[(size_t)p * 1056].data())};
            code_tokens(f, mbs, levels, p, nparts, w);
        } else {
            TokWriter w{e, probs};
            code_tokens(f, mbs, levels, p, nparts, w);
        }
        e.flush();
    });
    if (first_err) std::rethrow_exception(first_err);
    if (p1.size() >= (1u << 19)) throw std::runtime_error("vp8 writer: first partition too large");
    if (stats) {
        stats->n.assign(1056, std::array<uint32_t, 2>{0u, 0u});
        for (int p = 0; p < nparts; ++p)
            for (int k = 0; k < 1056; ++k) {
                stats->n[k][0] += cnt[(size_t)p * 1056 + k][0];
                stats->n[k][1] += cnt[(size_t)p * 1056 + k][1];
            }
        stats->valid = true;
        stats->us_first = job_us[0];
        stats->us_tokens = 0;
        for (int p = 0; p < nparts; ++p) stats->us_tokens += job_us[(size_t)p + 1];
    }
    // ---- assemble: frame tag, key-frame start code + size, partition 1, partition sizes, data
    const uint32_t tag = (f.key ? 0u : 1u) | (0u << 1) | (1u << 4) | ((uint32_t)p1.size() << 5);
    out.push_back((uint8_t)tag);
    out.push_back((uint8_t)(tag >> 8));
    out.push_back((uint8_t)(tag >> 16));
    if (f.key) {
        const uint8_t sc[3] = {0x9d, 0x01, 0x2a};
        out.insert(out.end(), sc, sc + 3);
        out.push_back((uint8_t)(f.width & 0xff));
        out.push_back((uint8_t)((f.width >> 8) & 0x3f));
        out.push_back((uint8_t)(f.height & 0xff));
        out.push_back((uint8_t)((f.height >> 8) & 0x3f));
    }
    out.insert(out.end(), p1.begin(), p1.end());
    for (int p = 0; p + 1 < nparts; ++p) {
        const uint32_t n = (uint32_t)parts[(size_t)p].size();
        out.push_back((uint8_t)n);
        out.push_back((uint8_t)(n >> 8));
        out.push_back((uint8_t)(n >> 16));
    }
    for (const auto& p : parts) out.insert(out.end(), p.begin(), p.end());
}

// ------------------------------------------------------------------ partition worker pool
PartitionPool::PartitionPool(int n) {
    for (int i = 0; i < n; ++i)
        th_.emplace_back([this]() {
            std::unique_lock<std::mutex> lk(mu_);
            for (;;) {
                cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
                if (stop_) return;
                Job* j = jobs_.front();  // the oldest job with tasks left
                const int k = j->next++;
                if (j->next >= j->total) jobs_.pop_front();
                lk.unlock();
                (*j->fn)(k);
                lk.lock();
                if (++j->finished == j->total) done_cv_.notify_all();
            }
        });
}

PartitionPool::~PartitionPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
}

void PartitionPool::run(int n, const std::function<void(int)>& fn) {
    if (th_.empty() || n <= 1) {
        for (int k = 0; k < n; ++k) fn(k);
        return;
    }
    Job j;
    j.fn = &fn;
    j.total = n;
    std::unique_lock<std::mutex> lk(mu_);
    jobs_.push_back(&j);
    cv_.notify_all();
    while (j.next < j.total) {  // the caller works on its own job too (it is awake already)
        const int k = j.next++;
        if (j.next >= j.total) jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &j));
        lk.unlock();
        fn(k);
        lk.lock();
        ++j.finished;
    }
    done_cv_.wait(lk, [&] { return j.finished == j.total; });
}

}  // namespace vp8
}  // namespace mx
