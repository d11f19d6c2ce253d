// HEVC host side: parameter sets / slice headers / Annex-B assembly (shared with the GPU
// encoder) and the serial CPU encoder, which makes exactly the decisions of the HIP
// kernels (hevc_kernels.hip) through the shared hevc_core.h functions.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "h264_mb.h"
#include "hevc_encoder.h"

namespace mx {
namespace hevc {

// ------------------------------------------------------------------ bit writer (headers)
namespace {
struct Bits {
    std::vector<uint8_t> b;
    uint32_t acc = 0;
    int n = 0;
    void put(uint32_t v, int k) {
        for (int i = k - 1; i >= 0; --i) {
            acc = (acc << 1) | ((v >> i) & 1);
            if (++n == 8) {
                b.push_back((uint8_t)acc);
                acc = 0;
                n = 0;
            }
        }
    }
    void ue(uint32_t v) {
        const uint64_t x = (uint64_t)v + 1;
        int len = 0;
        while ((x >> len) > 1) ++len;
        put(0, len);
        put((uint32_t)x, len + 1);
    }
    void se(int v) { ue(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
    void trailing() {  // rbsp_trailing_bits / byte_alignment: 1 then zeros
        put(1, 1);
        while (n) put(0, 1);
    }
};

void profile_tier_level(Bits& w, int level_idc) {
    w.put(0, 2);   // general_profile_space
    w.put(0, 1);   // general_tier_flag (Main tier)
    w.put(1, 5);   // general_profile_idc = Main
    w.put(0x60000000u, 32);  // compatibility flags 1 (Main) and 2 (Main 10)
    w.put(1, 1);   // progressive_source
    w.put(0, 1);   // interlaced_source
    w.put(1, 1);   // non_packed_constraint (no frame-packing SEI): codec string hvc1.1.6.Lxx.B0
    w.put(1, 1);   // frame_only_constraint
    w.put(0, 32);  // 43 reserved zero bits + general_inbld_flag
    w.put(0, 12);
    w.put((uint32_t)level_idc, 8);
}

void nal(std::vector<uint8_t>& out, int type, const std::vector<uint8_t>& rbsp) {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back((uint8_t)(type << 1));  // forbidden 0, nal_unit_type, nuh_layer_id high bit 0
    out.push_back(1);                      // nuh_layer_id low bits 0, nuh_temporal_id_plus1 = 1
    h264::emulation_prevent(out, rbsp.data(), rbsp.size());
}
}  // namespace

// Table A.6 (Main tier): general_level_idc, MaxLumaPs, MaxLumaSr, MaxSliceSegmentsPerPicture
struct LevelLimits {
    int idc;
    int64_t ps, sr;
    int slices;
};
static const LevelLimits kLevels[] = {
    {30, 36864, 552960, 16},           {60, 122880, 3686400, 16},          {63, 245760, 7372800, 20},
    {90, 552960, 16588800, 30},        {93, 983040, 33177600, 40},         {120, 2228224, 66846720, 75},
    {123, 2228224, 133693440, 75},     {150, 8912896, 267386880, 200},     {153, 8912896, 534773760, 200},
    {156, 8912896, 1069547520, 200},   {180, 35651584, 1069547520, 600},   {183, 35651584, 2139095040, 600},
    {186, 35651584, 4278190080LL, 600}};

int pick_level(int width, int height, int fps) {
    const int64_t ps = (int64_t)width * height, sr = ps * std::max(1, fps);
    for (const auto& l : kLevels) {
        const double maxdim = std::sqrt((double)l.ps * 8);
        if (ps <= l.ps && sr <= l.sr && width <= maxdim && height <= maxdim) return l.idc;
    }
    return 186;
}

int max_slices_for_level(int level_idc) {
    for (const auto& l : kLevels)
        if (l.idc == level_idc) return l.slices;
    return 600;
}

HevcCommon::HevcCommon(const EncoderConfig& c) : rc_(c) {
    level_ = pick_level(c.width, c.height, c.fps);
    const int maxs = max_slices_for_level(level_);
    slice_rows_ = 1;
    while ((c32_h() + slice_rows_ - 1) / slice_rows_ > maxs) ++slice_rows_;
    // two I slices per CTB row when the level allows: each intra wavefront then runs over half a
    // row (the 4K IDR's chain of 242 unit steps becomes 122, profiles/r05_SUMMARY.md)
    const int rows = (c32_h() + slice_rows_ - 1) / slice_rows_;
    i_split_ = (!c.hevc_wpp && c32_w() >= 2 && 2 * rows <= std::min(maxs, kMaxSlices)) ? 2 : 1;  // (WPP: row substreams)
    if (num_slices() > kMaxSlices) throw std::invalid_argument("hevc: too many slices");
    max_slices_ = std::min({maxs, kMaxSlices, num_ctbs()});
}

std::vector<int> HevcCommon::row_slices() const {
    std::vector<int> f;
    for (int s = 0; s < num_slices(); ++s) f.push_back((s / i_split_) * slice_rows_ * c32_w() + (s % i_split_) * (i_seg_w() / 2));
    return f;
}

std::vector<int> HevcCommon::plan_p_slices(const std::vector<CuInfo>& cus) const {
    if (wpp()) {  // slices of wpp_rows() CTB rows, one substream per CTB row
        std::vector<int> f;
        for (int y = 0; y < c32_h(); y += wpp_rows()) f.push_back(y * c32_w());
        return f;
    }
    // the cost of a CTB: the sum over its units
    std::vector<uint32_t> cc((size_t)num_ctbs(), 0u);
    for (int y = 0; y < ctb_h(); ++y)
        for (int x = 0; x < ctb_w(); ++x) cc[(size_t)ctb_of(x, y, c32_w())] += cu_cost(cus[(size_t)(y * ctb_w() + x)]);
    uint64_t total = 0;
    for (uint32_t v : cc) total += v;
    const int S = plan_num_slices(total, max_slices_, (uint32_t)rc_.config().hevc_slice_cost);
    std::vector<int> f;
    uint64_t pre = 0;
    int prev = -1;
    for (size_t i = 0; i < cc.size(); ++i) {
        const int id = plan_slice_of(pre, total, S);
        if (id != prev) f.push_back((int)i);
        prev = id;
        pre += cc[i];
    }
    return f;
}

void HevcCommon::write_parameter_sets(std::vector<uint8_t>& out) const {
    const EncoderConfig& c = config();
    const int cw = ctb_w() * kCtb, ch = ctb_h() * kCtb;
    {  // VPS
        Bits w;
        w.put(0, 4);       // vps_video_parameter_set_id
        w.put(1, 1);       // vps_base_layer_internal_flag
        w.put(1, 1);       // vps_base_layer_available_flag
        w.put(0, 6);       // vps_max_layers_minus1
        w.put(0, 3);       // vps_max_sub_layers_minus1
        w.put(1, 1);       // vps_temporal_id_nesting_flag
        w.put(0xffff, 16);
        profile_tier_level(w, level_);
        w.put(1, 1);  // vps_sub_layer_ordering_info_present_flag
        w.ue(1);      // vps_max_dec_pic_buffering_minus1
        w.ue(0);      // vps_max_num_reorder_pics
        w.ue(0);      // vps_max_latency_increase_plus1
        w.put(0, 6);  // vps_max_layer_id
        w.ue(0);      // vps_num_layer_sets_minus1
        w.put(0, 1);  // vps_timing_info_present_flag
        w.put(0, 1);  // vps_extension_flag
        w.trailing();
        nal(out, 32, w.b);
    }
    {  // SPS
        Bits w;
        w.put(0, 4);  // sps_video_parameter_set_id
        w.put(0, 3);  // sps_max_sub_layers_minus1
        w.put(1, 1);  // sps_temporal_id_nesting_flag
        profile_tier_level(w, level_);
        w.ue(0);  // sps_seq_parameter_set_id
        w.ue(1);  // chroma_format_idc 4:2:0
        w.ue((uint32_t)cw);
        w.ue((uint32_t)ch);
        const bool crop = cw != c.width || ch != c.height;
        w.put(crop, 1);
        if (crop) {
            w.ue(0);
            w.ue((uint32_t)(cw - c.width) / 2);
            w.ue(0);
            w.ue((uint32_t)(ch - c.height) / 2);
        }
        w.ue(0);  // bit_depth_luma_minus8
        w.ue(0);  // bit_depth_chroma_minus8
        w.ue(4);  // log2_max_pic_order_cnt_lsb_minus4 (8-bit POC LSB)
        w.put(1, 1);  // sps_sub_layer_ordering_info_present_flag
        w.ue(1);
        w.ue(0);
        w.ue(0);
        w.ue(kMinCbLog2 - 3);          // log2_min_luma_coding_block_size_minus3 (16)
        w.ue(kCtbLog2 - kMinCbLog2);   // log2_diff_max_min_luma_coding_block_size (CTB 32)
        w.ue(0);  // log2_min_luma_transform_block_size_minus2 (4)
        w.ue(kMaxTbLog2 - 2);  // log2_diff_max_min_luma_transform_block_size (16)
        w.ue((uint32_t)depth_inter());  // max_transform_hierarchy_depth_inter
        w.ue((uint32_t)depth_intra());  // max_transform_hierarchy_depth_intra
        w.put(0, 1);  // scaling_list_enabled_flag
        w.put(0, 1);  // amp_enabled_flag
        w.put(c.sao ? 1 : 0, 1);  // sample_adaptive_offset_enabled_flag
        w.put(0, 1);  // pcm_enabled_flag
        w.ue(1);      // num_short_term_ref_pic_sets
        w.ue(1);      // st_ref_pic_set(0): num_negative_pics
        w.ue(0);      //   num_positive_pics
        w.ue(0);      //   delta_poc_s0_minus1
        w.put(1, 1);  //   used_by_curr_pic_s0_flag
        w.put(0, 1);  // long_term_ref_pics_present_flag
        w.put(0, 1);  // sps_temporal_mvp_enabled_flag
        w.put(0, 1);  // strong_intra_smoothing_enabled_flag
        w.put(1, 1);  // vui_parameters_present_flag
        w.put(0, 1);  //   aspect_ratio_info_present_flag
        w.put(0, 1);  //   overscan_info_present_flag
        w.put(1, 1);  //   video_signal_type_present_flag
        w.put(5, 3);  //     video_format (unspecified)
        w.put(0, 1);  //     video_full_range_flag (limited range, as the CSC produces)
        w.put(1, 1);  //     colour_description_present_flag
        w.put(1, 8);  //     colour_primaries BT.709
        w.put(1, 8);  //     transfer_characteristics BT.709
        w.put(1, 8);  //     matrix_coeffs BT.709
        w.put(0, 1);  //   chroma_loc_info_present_flag
        w.put(0, 1);  //   neutral_chroma_indication_flag
        w.put(0, 1);  //   field_seq_flag
        w.put(0, 1);  //   frame_field_info_present_flag
        w.put(0, 1);  //   default_display_window_flag
        w.put(1, 1);  //   vui_timing_info_present_flag
        w.put(1, 32);  //     vui_num_units_in_tick
        w.put((uint32_t)std::max(1, c.fps), 32);  // vui_time_scale
        w.put(0, 1);  //     vui_poc_proportional_to_timing_flag
        w.put(0, 1);  //     vui_hrd_parameters_present_flag
        w.put(0, 1);  //   bitstream_restriction_flag
        w.put(0, 1);  // sps_extension_present_flag
        w.trailing();
        nal(out, 33, w.b);
    }
    {  // PPS
        Bits w;
        w.ue(0);      // pps_pic_parameter_set_id
        w.ue(0);      // pps_seq_parameter_set_id
        w.put(0, 1);  // dependent_slice_segments_enabled_flag
        w.put(0, 1);  // output_flag_present_flag
        w.put(0, 3);  // num_extra_slice_header_bits
        w.put(0, 1);  // sign_data_hiding_enabled_flag
        w.put(0, 1);  // cabac_init_present_flag
        w.ue(0);      // num_ref_idx_l0_default_active_minus1
        w.ue(0);      // num_ref_idx_l1_default_active_minus1
        w.se(0);      // init_qp_minus26
        w.put(0, 1);  // constrained_intra_pred_flag
        w.put(0, 1);  // transform_skip_enabled_flag
        w.put(1, 1);  // cu_qp_delta_enabled_flag
        w.ue(kCtbLog2 - 4);  // diff_cu_qp_delta_depth: 16x16 quantization groups
        w.se(c.chroma_qp_offset);  // pps_cb_qp_offset
        w.se(c.chroma_qp_offset);  // pps_cr_qp_offset
        w.put(0, 1);  // pps_slice_chroma_qp_offsets_present_flag
        w.put(0, 1);  // weighted_pred_flag
        w.put(0, 1);  // weighted_bipred_flag
        w.put(0, 1);  // transquant_bypass_enabled_flag
        w.put(0, 1);  // tiles_enabled_flag
        w.put(wpp() ? 1 : 0, 1);  // entropy_coding_sync_enabled_flag
        const bool db = c.hevc_deblock();
        w.put(db || c.sao, 1);  // pps_loop_filter_across_slices_enabled_flag (CU edges on slice borders too)
        w.put(1, 1);   // deblocking_filter_control_present_flag
        w.put(c.hevc_deblock_auto(), 1);  //   deblocking_filter_override_enabled_flag (adaptive: per slice)
        w.put(!db, 1);  //   pps_deblocking_filter_disabled_flag
        if (db) {
            w.se(0);  //   pps_beta_offset_div2
            w.se(0);  //   pps_tc_offset_div2
        }
        w.put(0, 1);  // pps_scaling_list_data_present_flag
        w.put(0, 1);  // lists_modification_present_flag
        w.ue(0);      // log2_parallel_merge_level_minus2
        w.put(0, 1);  // slice_segment_header_extension_present_flag
        w.put(0, 1);  // pps_extension_present_flag
        w.trailing();
        nal(out, 34, w.b);
    }
}

void HevcCommon::write_slice_nal(std::vector<uint8_t>& out, int addr, bool idr, int poc, int qp, bool deblock,
                                 const uint8_t* data, size_t n, const uint32_t* sub_len, int nsub,
                                 const uint32_t* sub_off) const {
    const int ctbs = num_ctbs();
    Bits w;
    w.put(addr == 0, 1);  // first_slice_segment_in_pic_flag
    if (idr) w.put(0, 1);  // no_output_of_prior_pics_flag
    w.ue(0);               // slice_pic_parameter_set_id
    if (addr != 0) {
        int bits = 0;
        while ((1 << bits) < ctbs) ++bits;
        w.put((uint32_t)addr, bits);  // slice_segment_address
    }
    w.ue(idr ? 2 : 1);  // slice_type I / P
    if (!idr) {
        w.put((uint32_t)(poc & 255), 8);  // slice_pic_order_cnt_lsb
        w.put(1, 1);                      // short_term_ref_pic_set_sps_flag
    }
    const bool sao = config().sao != 0;
    if (sao) {
        w.put(1, 1);  // slice_sao_luma_flag
        w.put(1, 1);  // slice_sao_chroma_flag
    }
    if (!idr) {
        w.put(0, 1);  // num_ref_idx_active_override_flag
        w.ue(5 - kMaxMergeCand);  // five_minus_max_num_merge_cand -> MaxNumMergeCand 5
    }
    w.se(qp - 26);  // slice_qp_delta
    if (config().hevc_deblock_auto()) {  // adaptive filter: override the PPS (filter on) where it is off
        w.put(!deblock, 1);       // deblocking_filter_override_flag
        if (!deblock) w.put(1, 1);  // slice_deblocking_filter_disabled_flag
    }
    if ((config().hevc_deblock() || sao) && (sao || deblock))
        w.put(1, 1);  // slice_loop_filter_across_slices_enabled_flag
    if (!wpp()) {
        w.trailing();   // byte_alignment()
        std::vector<uint8_t> rbsp = std::move(w.b);
        rbsp.insert(rbsp.end(), data, data + n);
        nal(out, idr ? 19 : 1, rbsp);  // IDR_W_RADL / TRAIL_R
        return;
    }
    // entry points: every substream ends in a byte holding its alignment one-bit, so emulation
    // prevention never spans two substreams and each can be escaped on its own
    std::vector<uint8_t> esc;
    std::vector<uint32_t> esc_len;
    size_t at = 0, total = 0;
    for (int k = 0; k < nsub; ++k) {
        const size_t before = esc.size();
        if (sub_off) at = sub_off[k];
        h264::emulation_prevent(esc, data + at, sub_len[k]);
        esc_len.push_back((uint32_t)(esc.size() - before));
        at += sub_len[k];
        total += sub_len[k];
    }
    if (total != n) throw std::logic_error("hevc: substream sizes do not add up to the slice payload");
    w.ue((uint32_t)(nsub > 0 ? nsub - 1 : 0));  // num_entry_point_offsets
    if (nsub > 1) {
        uint32_t mx = 0;
        for (int k = 0; k + 1 < nsub; ++k) mx = std::max(mx, esc_len[k] - 1);
        int len = 1;
        while (len < 32 && (mx >> len)) ++len;
        w.ue((uint32_t)(len - 1));  // offset_len_minus1
        for (int k = 0; k + 1 < nsub; ++k) w.put(esc_len[k] - 1, len);  // entry_point_offset_minus1
    }
    w.trailing();  // byte_alignment()
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back((uint8_t)((idr ? 19 : 1) << 1));
    out.push_back(1);
    h264::emulation_prevent(out, w.b.data(), w.b.size());  // the header ends in its alignment one-bit too
    out.insert(out.end(), esc.begin(), esc.end());
}

uint32_t code_slice_wpp(uint8_t* out, uint32_t cap, bool islice, int slice_qp, const PicSyn& ps, int first, int end,
                        uint16_t* tok, std::vector<uint32_t>& sub_len) {
    sub_len.clear();
    const int cw = ctb_cols(ps.mb_w);
    uint8_t ctx[C_NUM], saved[C_NUM];
    bool have_saved = false;
    uint32_t pos = 0;
    CabacEnc e;
    ArrCtx cx{ctx};
    for (int c = first; c < end; ++c) {
        const int x = c % cw;
        if (c == first || x == 0) {  // a substream starts
            if (c > first && have_saved && cw >= 2)
                std::memcpy(ctx, saved, C_NUM);  // sync from the row above after its second CTB (9.3.2.4)
            else
                ctx_init_all(ctx, islice ? 0 : 1, slice_qp);
            have_saved = false;
            e.start(out + pos, cap > pos ? cap - pos : 0);
        }
        code_ctb(e, cx, ps, islice, c, first, end, true, tok, false);
        if (x == 1) {  // storage after the row's second CTB (9.3.2.2 end)
            std::memcpy(saved, ctx, C_NUM);
            have_saved = true;
        }
        if (c == end - 1 || x == cw - 1) {  // substream ends: end_of_slice / end_of_subset coded
            e.finish_slice();
            if (e.overflow) return cap + 1;
            sub_len.push_back(e.pos);
            pos += e.pos;
        }
    }
    return pos;
}

// ------------------------------------------------------------------ CPU encoder
CpuHevcEncoder::CpuHevcEncoder(const EncoderConfig& cfg) : cfg_(cfg.with_aq_default(6)), common_(cfg) {
    cw_ = common_.ctb_w() * kCtb;
    ch_ = common_.ctb_h() * kCtb;
    for (int i = 0; i < 2; ++i) {
        rec_y_[i].assign((size_t)cw_ * ch_, 16);
        rec_uv_[i].assign((size_t)cw_ * ch_ / 2, 128);
    }
    const size_t n = (size_t)common_.ctb_w() * common_.ctb_h();
    cu_.resize(n);
    mv_.resize(2 * n);
    coef_.resize(n * kCoefPerCu);
    qp_pred_.assign(n, 0);
    qpy_.assign(n, 0);
    bl_safe_ = bl_safe_modes(4, 0) & bl_safe_modes(3, 1);  // the 16x16 luma mode and its DM chroma
    bl_safe_split_ = bl_safe_split();
}

namespace {
// Finish a CU's residual bookkeeping: cbf / last / coded sub-block masks.
void summarise(CuInfo& c, const int16_t* coef) {
    cu_summarise(c, coef);
    set_est_bytes(c, cu_bits_est(coef, c.tu_split == 2, c.tu4));
}

// 4x4 Hadamard SATD of the 16x16 source block at (x0, y0) against pred (raster 16x16): the sum over
// its sixteen 4x4 blocks (k_hevc_intra_modes: the same sums on the matrix cores).
int satd16(const uint8_t* sy, int pitch, int x0, int y0, const int* pred) {
    int satd = 0;
    for (int by = 0; by < 16; by += 4)
        for (int bx = 0; bx < 16; bx += 4) {
            int d[4][4], h[4][4];
            for (int r = 0; r < 4; ++r)
                for (int q = 0; q < 4; ++q)
                    d[r][q] = (int)sy[(size_t)(y0 + by + r) * pitch + x0 + bx + q] - pred[(by + r) * 16 + bx + q];
            for (int r = 0; r < 4; ++r) {  // rows, then columns: 4-point Walsh-Hadamard
                const int a0 = d[r][0] + d[r][1], a1 = d[r][0] - d[r][1], a2 = d[r][2] + d[r][3], a3 = d[r][2] - d[r][3];
                h[r][0] = a0 + a2;
                h[r][1] = a1 + a3;
                h[r][2] = a0 - a2;
                h[r][3] = a1 - a3;
            }
            for (int q = 0; q < 4; ++q) {
                const int a0 = h[0][q] + h[1][q], a1 = h[0][q] - h[1][q], a2 = h[2][q] + h[3][q], a3 = h[2][q] - h[3][q];
                satd += std::abs(a0 + a2) + std::abs(a1 + a3) + std::abs(a0 - a2) + std::abs(a1 - a3);
            }
        }
    return satd;
}

// Substituted references (intra_refs) of the N x N block at (x, y) of a plane -- step 1: luma, 2: one
// NV12 chroma component (p at its first sample) -- with availability avl (split_tu_avl bits).
void block_refs(const uint8_t* p, int pitch, int step, int x, int y, int N, int avl, int* L, int* T) {
    uint8_t lp[16], bp[16], tp[16], tr[16];
    auto px = [&](int xx, int yy) { return p[(size_t)yy * pitch + (size_t)xx * step]; };
    for (int k = 0; k < N; ++k) {
        lp[k] = (avl & 2) ? px(x - 1, y + k) : 0;
        bp[k] = (avl & 1) ? px(x - 1, y + N + k) : 0;
        tp[k] = (avl & 8) ? px(x + k, y - 1) : 0;
        tr[k] = (avl & 16) ? px(x + N + k, y - 1) : 0;
    }
    const int corner = (avl & 4) ? px(x - 1, y - 1) : 0;
    intra_refs(N, (avl & 2) != 0, (avl & 1) != 0, (avl & 8) != 0, (avl & 16) != 0, (avl & 4) != 0, lp, bp, tp, tr,
               corner, L, T);
}
}  // namespace

// Open-loop intra mode of the 16x16 unit (x, y) of a picture of mb_w x mb_h units in I slices of
// sr unit rows (k_hevc_intra_modes on the GPU): all 35 modes predicted from the *source*
// neighbours with the decoder's z-order availability (never the below-left; a CTB's first unit only
// uses the modes in `safe` -- bl_safe_modes -- because the raster wavefront reconstructs it before
// its below-left), scored by the 4x4 Hadamard SATD of the residual + lambda * mode bits, searched
// coarse-to-fine (intra_mode_search: at most 15 of the 35 modes); the lowest cost wins, ties to the
// lower mode.  With split, the modes are searched again (same order) for the unit predicted as four
// 8x8 TUs from the source (split_tu_avl; a CTB's first unit only in safe_split modes), and that mode
// with kIntraSplitFlag wins when intra_split_wins over the unsplit cost (mode bits included).
int intra_decide_mode(const uint8_t* sy, int pitch, int mb_w, int mb_h, int x, int y, int sr, int seg_w, int qp,
                      uint64_t safe, uint64_t safe_split, bool split) {
    const int x0 = x * 16, y0 = y * 16, z = ((y & 1) << 1) | (x & 1);
    int xb, xe;
    i_seg_range(x, seg_w, mb_w, xb, xe);
    const bool al = x > xb, at = (y % sr) != 0, atr = at && x + 1 < xe && z != 3, ac = at && x > xb;
    const bool bl_pending = z == 0 && x > xb && y + 1 < mb_h;
    uint8_t lp[16], tp[16], tr[16];
    for (int k = 0; k < 16; ++k) {
        lp[k] = al ? sy[(size_t)(y0 + k) * pitch + x0 - 1] : 0;
        tp[k] = at ? sy[(size_t)(y0 - 1) * pitch + x0 + k] : 0;
        tr[k] = atr ? sy[(size_t)(y0 - 1) * pitch + x0 + 16 + k] : 0;
    }
    const int corner = ac ? sy[(size_t)(y0 - 1) * pitch + x0 - 1] : 0;
    int L[33], T[33], pred[256];
    intra_refs(16, al, false, at, atr, ac, lp, lp, tp, tr, corner, L, T);
    const int lambda = h264::lambda_sad(qp);
    auto cost = [&](int m) {
        if (bl_pending && !((safe >> m) & 1)) return kIntraNoMode;
        intra_predict(m, 4, 0, L, T, pred);
        return satd16(sy, pitch, x0, y0, pred) + lambda * intra_mode_bits(m, 1, 1);
    };
    const int best = intra_mode_search(cost);
    if (!split || !intra_split_possible(cost(best), lambda)) return best;
    int Lk[4][17], Tk[4][17];
    for (int k = 0; k < 4; ++k)
        block_refs(sy, pitch, 1, x0 + (k & 1) * 8, y0 + (k >> 1) * 8, 8, split_tu_avl(k, al, ac, at, atr), Lk[k], Tk[k]);
    auto cost_split = [&](int m) {
        if (bl_pending && !((safe_split >> m) & 1)) return kIntraNoMode;
        for (int k = 0; k < 4; ++k) {
            const int bx = (k & 1) * 8, by = (k >> 1) * 8;
            int p8[64];
            intra_predict(m, 3, 0, Lk[k], Tk[k], p8);
            for (int r = 0; r < 8; ++r)
                for (int q = 0; q < 8; ++q) pred[(by + r) * 16 + bx + q] = p8[r * 8 + q];
        }
        return satd16(sy, pitch, x0, y0, pred) + lambda * intra_mode_bits(m, 1, 1);
    };
    const int best_s = intra_mode_search(cost_split);
    return intra_split_wins(cost(best), cost_split(best_s), lambda) ? best_s | kIntraSplitFlag : best;
}

void CpuHevcEncoder::analyse_intra(const uint8_t* sy, const uint8_t* suv, int pitch) {
    uint8_t* ry = rec_y_[cur_].data();
    uint8_t* ruv = rec_uv_[cur_].data();
    const int W = common_.ctb_w(), H = common_.ctb_h(), sr = 2 * common_.slice_rows();  // unit rows per I slice
    const int qp = frame_qp_();
    const int qpc = chroma_qp(qp, cfg_.chroma_qp_offset);
    const bool split_on = common_.depth_intra() > 0;
    // units in raster order (the GPU's row wavefront) with the modes decided open-loop on the
    // source (intra_decide_mode); availability as the decoder sees it in z order: no above-right
    // for a CTB's last unit, no below-left reads by a CTB's first unit (see bl_safe_modes)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int i = y * W + x, x0 = x * 16, y0 = y * 16;
            const int z = ((y & 1) << 1) | (x & 1);
            CuInfo& c = cu_[i];
            std::memset(&c, 0, sizeof c);
            int xb, xe;
            i_seg_range(x, common_.i_seg_w(), W, xb, xe);
            const bool al = x > xb, at = (y % sr) != 0, atr = at && x + 1 < xe && z != 3, ac = at && x > xb;
            const int dm = intra_decide_mode(sy, pitch, W, H, x, y, sr, common_.i_seg_w(), qp, bl_safe_, bl_safe_split_,
                                             split_on);
            const int best = dm & (kIntraSplitFlag - 1);
            c.type = kCuIntra;
            c.intra_mode = (uint8_t)best;
            c.qp = (uint8_t)qp;
            c.ct = 1;
            int16_t* co = coef_.data() + (size_t)i * kCoefPerCu;
            if (dm & kIntraSplitFlag) {
                // four 8x8 luma TUs, then per TU its two 4x4 chroma TUs, each predicted from the
                // reconstruction so far (ry / ruv hold it as the TUs complete)
                c.tu_split = 2;
                const int scan = intra_scan_idx(best);
                for (int k = 0; k < 4; ++k) {
                    const int avl = split_tu_avl(k, al, ac, at, atr);
                    const int bx = x0 + (k & 1) * 8, by = y0 + (k >> 1) * 8;
                    int Lk[17], Tk[17], p8[64], r8[64], rr8[64];
                    block_refs(ry, cw_, 1, bx, by, 8, avl, Lk, Tk);
                    intra_predict(best, 3, 0, Lk, Tk, p8);
                    for (int r = 0; r < 8; ++r)
                        for (int q = 0; q < 8; ++q) r8[r * 8 + q] = sy[(size_t)(by + r) * pitch + bx + q] - p8[r * 8 + q];
                    tu_encode(3, r8, qp, true, co + 64 * k, rr8, scan);
                    for (int r = 0; r < 8; ++r)
                        for (int q = 0; q < 8; ++q) ry[(by + r) * cw_ + bx + q] = (uint8_t)clip255(p8[r * 8 + q] + rr8[r * 8 + q]);
                    const int cx = bx / 2, cy = by / 2;
                    for (int comp = 0; comp < 2; ++comp) {
                        int Lc[9], Tc[9], p4[16], r4[16], rr4[16];
                        block_refs(ruv + comp, cw_, 2, cx, cy, 4, avl, Lc, Tc);
                        intra_predict(best, 2, 1 + comp, Lc, Tc, p4);
                        for (int r = 0; r < 4; ++r)
                            for (int q = 0; q < 4; ++q)
                                r4[r * 4 + q] = suv[(size_t)(cy + r) * pitch + 2 * (cx + q) + comp] - p4[r * 4 + q];
                        tu_encode(2, r4, qpc, true, co + 256 + 64 * comp + 16 * k, rr4, scan);
                        for (int r = 0; r < 4; ++r)
                            for (int q = 0; q < 4; ++q)
                                ruv[(cy + r) * cw_ + 2 * (cx + q) + comp] = (uint8_t)clip255(p4[r * 4 + q] + rr4[r * 4 + q]);
                    }
                }
                summarise(c, co);
                mv_[2 * i] = mv_[2 * i + 1] = 0;
                continue;
            }
            uint8_t lp[16], tp[16], tr[16];
            for (int k = 0; k < 16; ++k) {
                lp[k] = al ? ry[(y0 + k) * cw_ + x0 - 1] : 0;
                tp[k] = at ? ry[(y0 - 1) * cw_ + x0 + k] : 0;
                tr[k] = atr ? ry[(y0 - 1) * cw_ + x0 + 16 + k] : 0;
            }
            const int corner = ac ? ry[(y0 - 1) * cw_ + x0 - 1] : 0;
            int L[33], T[33];
            intra_refs(16, al, false, at, atr, ac, lp, lp, tp, tr, corner, L, T);
            int pred[256];
            intra_predict(best, 4, 0, L, T, pred);
            int res[256], rr[256];
            for (int r = 0; r < 16; ++r)
                for (int q = 0; q < 16; ++q) res[r * 16 + q] = sy[(y0 + r) * pitch + x0 + q] - pred[r * 16 + q];
            tu_encode(4, res, qp, true, co, rr);
            for (int r = 0; r < 16; ++r)
                for (int q = 0; q < 16; ++q) ry[(y0 + r) * cw_ + x0 + q] = (uint8_t)clip255(pred[r * 16 + q] + rr[r * 16 + q]);
            for (int comp = 0; comp < 2; ++comp) {
                const int xc = x0 / 2, yc = y0 / 2;
                uint8_t lc[8], tc[8], trc[8];
                for (int k = 0; k < 8; ++k) {
                    lc[k] = al ? ruv[(yc + k) * cw_ + 2 * (xc - 1) + comp] : 0;
                    tc[k] = at ? ruv[(yc - 1) * cw_ + 2 * (xc + k) + comp] : 0;
                    trc[k] = atr ? ruv[(yc - 1) * cw_ + 2 * (xc + 8 + k) + comp] : 0;
                }
                const int cc = ac ? ruv[(yc - 1) * cw_ + 2 * (xc - 1) + comp] : 0;
                int Lc[17], Tc[17], pc[64], rc[64], rrc[64];
                intra_refs(8, al, false, at, atr, ac, lc, lc, tc, trc, cc, Lc, Tc);
                intra_predict(best, 3, 1 + comp, Lc, Tc, pc);
                for (int r = 0; r < 8; ++r)
                    for (int q = 0; q < 8; ++q) rc[r * 8 + q] = suv[(yc + r) * pitch + 2 * (xc + q) + comp] - pc[r * 8 + q];
                tu_encode(3, rc, qpc, true, co + 256 + 64 * comp, rrc);
                for (int r = 0; r < 8; ++r)
                    for (int q = 0; q < 8; ++q)
                        ruv[(yc + r) * cw_ + 2 * (xc + q) + comp] = (uint8_t)clip255(pc[r * 8 + q] + rrc[r * 8 + q]);
            }
            summarise(c, co);
            mv_[2 * i] = mv_[2 * i + 1] = 0;
        }
}

void CpuHevcEncoder::analyse_inter(const uint8_t* sy, const uint8_t* suv, int pitch) {
    const uint8_t* ref_y = rec_y_[cur_ ^ 1].data();
    const uint8_t* ref_uv = rec_uv_[cur_ ^ 1].data();
    uint8_t* ry = rec_y_[cur_].data();
    uint8_t* ruv = rec_uv_[cur_].data();
    const int W = common_.ctb_w(), H = common_.ctb_h(), sr = common_.slice_rows();
    const int fqp = frame_qp_();
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int i = y * W + x;
            int mvx = 0, mvy = 0;
            h264::me_search_cpu(sy, pitch, ref_y, cw_, ch_, x * 16, y * 16, fqp, cfg_.search_range, cfg_.subpel, &mvx,
                                &mvy, cfg_.me_coarse);
            mv_[2 * i] = (int16_t)mvx;
            mv_[2 * i + 1] = (int16_t)mvy;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int i = y * W + x, x0 = x * 16, y0 = y * 16;
            CuInfo& c = cu_[i];
            std::memset(&c, 0, sizeof c);
            c.mvx = mv_[2 * i];
            c.mvy = mv_[2 * i + 1];
            int pred[256], res[256], rr[256];
            uint32_t lsad = 0;
            for (int r = 0; r < 16; ++r)
                for (int q = 0; q < 16; ++q) {
                    const int p = luma_mc(ref_y, cw_, cw_, ch_, x0 + q, y0 + r, c.mvx, c.mvy);
                    pred[r * 16 + q] = p;
                    res[r * 16 + q] = sy[(y0 + r) * pitch + x0 + q] - p;
                    lsad += (uint32_t)std::abs(res[r * 16 + q]);
                }
            // temporal class (aq 3): the source's change against the previous source, displaced by
            // the integer part of the vector
            uint32_t tsad = 0;
            if (cfg_.aq >= 3 && !prev_src_.empty())
                for (int r = 0; r < 16; ++r)
                    for (int q = 0; q < 16; ++q)
                        tsad += (uint32_t)std::abs((int)sy[(y0 + r) * pitch + x0 + q] -
                                                   h264::ref_px(prev_src_.data(), cw_, cw_, ch_, x0 + q + (c.mvx >> 2),
                                                                y0 + r + (c.mvy >> 2)));
            const int tcls = h264::temporal_class(tsad, c.mvx == 0 && c.mvy == 0);
            const int qp = h264::mb_qp_for(fqp, lsad, tcls, cfg_.aq);
            const int qpc = chroma_qp(qp, cfg_.chroma_qp_offset);
            const bool changing = cfg_.aq >= 3 && tcls == h264::kTcChanging;
            c.qp = (uint8_t)qp;
            int16_t* co = coef_.data() + (size_t)i * kCoefPerCu;
            int pc[2][64], rc[2][64];
            const int xc = x0 / 2, yc = y0 / 2;
            for (int comp = 0; comp < 2; ++comp)
                for (int r = 0; r < 8; ++r)
                    for (int q = 0; q < 8; ++q) {
                        const int p = chroma_mc(ref_uv, cw_, cw_ / 2, ch_ / 2, comp, xc + q, yc + r, c.mvx, c.mvy);
                        pc[comp][r * 8 + q] = p;
                        rc[comp][r * 8 + q] = (changing && !cfg_.hevc_chroma_keep) ? 0 : suv[(yc + r) * pitch + 2 * (xc + q) + comp] - p;
                    }
            // option 1: one 16x16 luma TU, 8x8 chroma TUs
            int rrc[2][64];
            tu_encode(4, res, qp, false, co, rr);
            for (int comp = 0; comp < 2; ++comp) tu_encode(3, rc[comp], qpc, false, co + 256 + 64 * comp, rrc[comp]);
            c.tu_split = cfg_.tu_split ? 1 : 0;
            int levels1 = 0;
            for (int k = 0; k < kCoefPerCu; ++k) levels1 += co[k] != 0;
            c.tu4 = 0;
            if (cfg_.tu_split && split_worth_trying(levels1)) {
                // option 2: four 8x8 luma nodes (each one 8x8 TU or, tu_split 2, four 4x4 TUs), eight
                // 4x4 chroma TUs; keep the cheaper by SSE + lambda * bits
                int16_t co2[kCoefPerCu];
                int rr2[256], rrc2[2][64];
                const int tu4 = split_encode(res, rc, qp, qpc, co2, rr2, rrc2, pred, cfg_.tu_split >= 2);
                uint64_t sse1 = 0, sse2 = 0;
                for (int k = 0; k < 256; ++k) {
                    const int s0 = pred[k] + res[k];
                    const int e1 = s0 - clip255(pred[k] + rr[k]), e2 = s0 - clip255(pred[k] + rr2[k]);
                    sse1 += (uint64_t)(e1 * e1);
                    sse2 += (uint64_t)(e2 * e2);
                }
                for (int comp = 0; comp < 2; ++comp)
                    for (int k = 0; k < 64; ++k) {
                        const int s0 = pc[comp][k] + rc[comp][k];
                        const int e1 = s0 - clip255(pc[comp][k] + rrc[comp][k]);
                        const int e2 = s0 - clip255(pc[comp][k] + rrc2[comp][k]);
                        sse1 += (uint64_t)(e1 * e1);
                        sse2 += (uint64_t)(e2 * e2);
                    }
                if (choose_split(sse1, cu_bits_est(co, false), sse2, cu_bits_est(co2, true, tu4), qp)) {
                    c.tu_split = 2;
                    c.tu4 = (uint8_t)tu4;
                    std::memcpy(co, co2, sizeof co2);
                    std::memcpy(rr, rr2, sizeof rr2);
                    std::memcpy(rrc, rrc2, sizeof rrc2);
                }
            }
            if (changing && !cfg_.hevc_chroma_keep) {
                // rate-distortion residual drop (h264_mb.h drop_luma_for): the luma residual must
                // lower the distortion by more than lambda * (estimated bits of the chosen tree)
                long long d_pred = 0, d_coded = 0;
                for (int k = 0; k < 256; ++k) {
                    const int e = pred[k] + res[k] - clip255(pred[k] + rr[k]);
                    d_pred += res[k] * res[k];
                    d_coded += e * e;
                }
                const uint32_t bits = luma_bits_est(co, c.tu_split == 2, c.tu4);
                if (h264::drop_luma_for(cfg_.aq, lsad, tcls, qp, d_pred, d_coded, bits)) {
                    for (int k = 0; k < 256; ++k) co[k] = 0, rr[k] = 0;
                    c.tu_split = cfg_.tu_split ? 1 : 0;
                    c.tu4 = 0;
                }
            }
            for (int r = 0; r < 16; ++r)
                for (int q = 0; q < 16; ++q) ry[(y0 + r) * cw_ + x0 + q] = (uint8_t)clip255(pred[r * 16 + q] + rr[r * 16 + q]);
            for (int comp = 0; comp < 2; ++comp)
                for (int r = 0; r < 8; ++r)
                    for (int q = 0; q < 8; ++q)
                        ruv[(yc + r) * cw_ + 2 * (xc + q) + comp] =
                            (uint8_t)clip255(pc[comp][r * 8 + q] + rrc[comp][r * 8 + q]);
            summarise(c, co);
        }
    // cost-balanced slices of CTBs, then per CTB the skip / merge / AMVP decisions against the
    // slice's neighbours and the coding tree (CU32 or four CU16)
    slices_ = common_.plan_p_slices(cu_);
    const int cw = common_.c32_w(), nctb = common_.num_ctbs();
    for (size_t s = 0; s < slices_.size(); ++s) {
        const int first = slices_[s], end = s + 1 < slices_.size() ? slices_[s + 1] : nctb;
        for (int c = first; c < end; ++c) {
            const int x0 = 2 * (c % cw), y0 = 2 * (c / cw);
            CuInfo u[4];
            bool in[4];
            for (int z = 0; z < 4; ++z) {
                const int x = x0 + (z & 1), y = y0 + (z >> 1);
                in[z] = x < W && y < H;
                if (in[z]) u[z] = cu_[(size_t)(y * W + x)];
            }
            decide_ctb(u, in, mv_.data(), 2, x0, y0, W, H, first);
            for (int z = 0; z < 4; ++z)
                if (in[z]) cu_[(size_t)((y0 + (z >> 1)) * W + x0 + (z & 1))] = u[z];
        }
    }
    (void)sr;
}

const std::vector<uint8_t>& CpuHevcEncoder::encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr) {
    h264::EncoderCommon& rc = common_.rc();
    const int W = common_.ctb_w(), H = common_.ctb_h(), nctb = common_.num_ctbs();
    auto slice_end = [&](size_t s) { return s + 1 < slices_.size() ? slices_[s + 1] : nctb; };
    auto qp_chain = [&](int qp) {  // QP predictors / QpY of every unit, slice by slice
        for (size_t s = 0; s < slices_.size(); ++s)
            slice_qp_chain(cu_.data(), W, H, slices_[s], slice_end(s), qp, common_.wpp(), qp_pred_.data(), qpy_.data());
    };
    while (rc.wants_probe()) {  // size the first IDR (rate control), as the GPU encoder does
        qp_override_ = rc.probe_qp();
        analyse_intra(y, uv, pitch);
        slices_ = common_.row_slices();
        qp_chain(qp_override_);
        const PicSyn ps{cu_.data(), coef_.data(), qp_pred_.data(), nullptr, W, H, common_.depth_inter(),
                        common_.depth_intra()};
        std::vector<uint8_t> buf;
        std::vector<uint32_t> sub_len;
        uint8_t ctx[C_NUM];
        size_t total = 0;
        for (size_t s = 0; s < slices_.size(); ++s) {
            const int first = slices_[s], end = slice_end(s);
            const uint32_t cap = (uint32_t)(end - first) * 4096 + 1024;
            buf.resize(cap);
            total += (common_.wpp() ? code_slice_wpp(buf.data(), cap, true, qp_override_, ps, first, end, tok_.data(),
                                                     sub_len)
                                    : code_slice(buf.data(), cap, true, qp_override_, ps, first, end, ctx, tok_.data())) +
                     12;
        }
        rc.add_probe(qp_override_, (int)total + 64);
        qp_override_ = -1;
    }
    rc.begin_frame(force_idr || !have_ref_);
    const bool idr = rc.cur_idr();
    const int qp = rc.cur_qp();
    if (have_ref_) cur_ ^= 1;
    have_ref_ = true;
    if (idr) {
        analyse_intra(y, uv, pitch);
        slices_ = common_.row_slices();
    } else {
        analyse_inter(y, uv, pitch);
    }
    qp_chain(qp);
    deblock_now_ = cfg_.hevc_deblock();
    if (cfg_.hevc_deblock_auto()) {  // adaptive: k_hevc_db_auto's rule over the units' motion-search vectors
        if (!idr) {
            h264::DbAutoCounts c;
            for (int i = 0; i < W * H; ++i) h264::db_auto_count_mv(mv_.data(), 2, W, i, c);
            db_prev_on_ = h264::db_auto_decide(c, W * H, db_prev_on_);
        }
        deblock_now_ = db_prev_on_;
    }
    if (deblock_now_) {  // in-loop deblocking: all vertical edges, then all horizontal ones
        for (int dir = 0; dir < 2; ++dir)
            for (int i = 0; i < W * H; ++i)
                for (int seg = 0; seg < 4; ++seg) {
                    if (dir == 0 ? (i % W) != 0 : (i / W) != 0)
                        db_edge_seg(rec_y_[cur_].data(), rec_uv_[cur_].data(), cw_, W, cu_.data(), qpy_.data(), i, dir,
                                    seg, cfg_.chroma_qp_offset);
                    db_internal_seg(rec_y_[cur_].data(), cw_, W, cu_.data(), qpy_.data(), i, dir, seg);
                }
    }
    if (cfg_.sao) {  // SAO per 32x32 CTB on the deblocked picture (a copy: CTBs read deblocked neighbours)
        const std::vector<uint8_t> pre_y = rec_y_[cur_], pre_uv = rec_uv_[cur_];
        sao_.assign((size_t)nctb * 4, 0u);
        const uint32_t lam16 = kLambdaSse16[qp];
        const int cw = common_.c32_w();
        for (int c = 0; c < nctb; ++c) {
            const int x0 = (c % cw) * 32, y0 = (c / cw) * 32;
            const int nw = std::min(32, cw_ - x0), nh = std::min(32, ch_ - y0);
            uint32_t* w = sao_.data() + 4 * (size_t)c;
            uint32_t any = 0;
            for (int z = 0; z < 4; ++z) {
                const int ux = 2 * (c % cw) + (z & 1), uy = 2 * (c / cw) + (z >> 1);
                if (ux < W && uy < H) any |= cu_[(size_t)(uy * W + ux)].cbf;
            }
            if (!sao_keep_ctb(idr, any)) {
                SaoStats st[3];
                sao_stats_block(pre_y.data(), cw_, y, pitch, 1, x0, y0, nw, nh, cw_, ch_, st[0]);
                for (int k = 0; k < 2; ++k)
                    sao_stats_block(pre_uv.data() + k, cw_, uv + k, pitch, 2, x0 / 2, y0 / 2, nw / 2, nh / 2, cw_ / 2,
                                    ch_ / 2, st[1 + k]);
                SaoCompChoice ch[3];
                for (int k = 0; k < 3; ++k) sao_eval_comp(st[k], lam16, ch[k]);
                sao_combine(ch[0], ch[1], ch[2], lam16, w);
            }  // else SAO off, the samples are kept
            sao_apply_block(pre_y.data(), rec_y_[cur_].data(), cw_, 1, x0, y0, nw, nh, cw_, ch_, w[0]);
            for (int k = 0; k < 2; ++k)
                sao_apply_block(pre_uv.data() + k, rec_uv_[cur_].data() + k, cw_, 2, x0 / 2, y0 / 2, nw / 2, nh / 2,
                                cw_ / 2, ch_ / 2, w[1 + k]);
        }
    }
    au_.clear();
    if (idr) common_.write_parameter_sets(au_);
    std::vector<uint8_t> buf;
    std::vector<uint32_t> sub_len;
    uint8_t ctx[C_NUM];
    const PicSyn ps{cu_.data(), coef_.data(), qp_pred_.data(), cfg_.sao ? sao_.data() : nullptr, W, H,
                    common_.depth_inter(), common_.depth_intra()};
    for (size_t s = 0; s < slices_.size(); ++s) {
        const int first = slices_[s], end = slice_end(s);
        const uint32_t cap = (uint32_t)(end - first) * 4096 + 1024;
        buf.resize(cap);
        const uint32_t n = common_.wpp() ? code_slice_wpp(buf.data(), cap, idr, qp, ps, first, end, tok_.data(), sub_len)
                                         : code_slice(buf.data(), cap, idr, qp, ps, first, end, ctx, tok_.data());
        if (n > cap) throw std::runtime_error("hevc cpu encoder: slice buffer overflow");
        common_.write_slice_nal(au_, first, idr, idr ? 0 : common_.poc(), qp, deblock_now_, buf.data(), n,
                                common_.wpp() ? sub_len.data() : nullptr, (int)sub_len.size());
    }
    // distortion over the display area
    const EncoderConfig& c = common_.config();
    uint64_t sse[3] = {0, 0, 0};
    const uint8_t* ry = rec_y_[cur_].data();
    const uint8_t* ruv = rec_uv_[cur_].data();
    for (int r = 0; r < c.height; ++r)
        for (int q = 0; q < c.width; ++q) {
            const int d = (int)y[r * pitch + q] - ry[r * cw_ + q];
            sse[0] += (uint64_t)(d * d);
        }
    for (int r = 0; r < c.height / 2; ++r)
        for (int q = 0; q < c.width / 2; ++q)
            for (int comp = 0; comp < 2; ++comp) {
                const int d = (int)uv[r * pitch + 2 * q + comp] - ruv[r * cw_ + 2 * q + comp];
                sse[1 + comp] += (uint64_t)(d * d);
            }
    stats_.frame_index = rc.frames();
    stats_.idr = idr;
    stats_.qp = qp;
    stats_.bytes = (int)au_.size();
    stats_.deblocked = deblock_now_ ? 1 : 0;
    stats_.skipped_mbs = 0;
    for (const auto& cu : cu_) stats_.skipped_mbs += cu.type == kCuSkip;
    for (int k = 0; k < 3; ++k) stats_.sse[k] = sse[k];
    rc.end_frame((int)au_.size(), idr);
    if (cfg_.aq >= 3) {  // this frame's source becomes the previous source of the next one
        prev_src_.resize((size_t)cw_ * ch_);
        for (int r = 0; r < ch_; ++r) std::memcpy(prev_src_.data() + (size_t)r * cw_, y + (size_t)r * pitch, cw_);
    }
    return au_;
}

}  // namespace hevc
}  // namespace mx

namespace mx {
namespace hevc {

// Random slices (every CU type, CU32 and CU16 coding trees, split and unsplit transform trees,
// levels up to the escape range, SAO parameters) coded twice -- directly and through the
// bin-token path -- must give identical bytes.  Returns the number of slices checked; throws on
// the first mismatch.
int token_selftest(uint32_t seed, int slices) {
    uint32_t r = seed * 2654435761u + 1u;
    auto rnd = [&r](uint32_t n) {
        r ^= r << 13;
        r ^= r >> 17;
        r ^= r << 5;
        return n ? r % n : 0u;
    };
    for (int sl = 0; sl < slices; ++sl) {
        const int mb_w = 1 + (int)rnd(9), mb_h = 1 + (int)rnd(7);
        const int cw = ctb_cols(mb_w), nctb = cw * ctb_rows(mb_h);
        const int first = (int)rnd((uint32_t)nctb), end = first + 1 + (int)rnd((uint32_t)(nctb - first));
        const bool islice = rnd(4) == 0;
        const int qp = 10 + (int)rnd(40);
        const int nu = mb_w * mb_h;
        std::vector<CuInfo> cus((size_t)nu);
        std::vector<int16_t> coef((size_t)nu * kCoefPerCu, 0);
        std::vector<uint8_t> qpp((size_t)nu);
        std::vector<uint32_t> sao((size_t)nctb * 4, 0);
        auto fill_levels = [&](CuInfo& c, int i) {
            const int density = (int)rnd(4);  // 0: empty, 1: sparse, 2: dense, 3: escapes
            int16_t* co = coef.data() + (size_t)i * kCoefPerCu;
            for (int k = 0; k < kCoefPerCu && density; ++k) {
                if (rnd(density == 1 ? 40 : 3)) continue;
                int v = 1 + (int)rnd(density == 3 ? 3000 : 4);
                if (density == 3 && rnd(50) == 0) v = 30000;
                co[k] = (int16_t)(rnd(2) ? -v : v);
            }
            cu_summarise(c, co);
        };
        for (int c = 0; c < nctb; ++c) {
            const int x0 = 2 * (c % cw), y0 = 2 * (c / cw);
            const bool cu32 = !islice && ctb_whole(c, cw, mb_w, mb_h) && rnd(2);
            CuInfo h;
            std::memset(&h, 0, sizeof h);
            h.type = (uint8_t)rnd(3);  // skip / merge / AMVP
            h.qp = (uint8_t)(10 + rnd(40));
            h.mvx = (int16_t)((int)rnd(200) - 100);
            h.mvdx = (int16_t)((int)rnd(2000) - 1000);
            h.mvdy = (int16_t)((int)rnd(64) - 32);
            h.mvp_idx = (uint8_t)(h.type == kCuAmvp ? rnd(2) : rnd(5));
            for (int z = 0; z < 4; ++z) {
                const int x = x0 + (z & 1), y = y0 + (z >> 1);
                if (x >= mb_w || y >= mb_h) continue;
                const int i = y * mb_w + x;
                CuInfo& cu = cus[(size_t)i];
                std::memset(&cu, 0, sizeof cu);
                if (cu32) {
                    cu = h;
                    cu.ct = 0;
                } else {
                    cu.ct = 1;
                    cu.type = islice ? kCuIntra : (uint8_t)rnd(4);
                    cu.intra_mode = (uint8_t)rnd(35);
                    cu.qp = (uint8_t)(10 + rnd(40));
                    cu.mvdx = (int16_t)((int)rnd(2000) - 1000);
                    cu.mvdy = (int16_t)((int)rnd(64) - 32);
                    cu.mvp_idx = (uint8_t)(cu.type == kCuAmvp ? rnd(2) : rnd(5));
                }
                cu.tu_split = (uint8_t)(1 + rnd(2));  // intra too (max_transform_hierarchy_depth_intra 1 below)
                cu.tu4 = (cu.tu_split == 2 && cu.type != kCuIntra) ? (uint8_t)rnd(16) : 0;  // 8x8 nodes into 4x4 TUs
                if (cu.type != kCuSkip) fill_levels(cu, i);
                qpp[(size_t)i] = (uint8_t)(10 + rnd(40));
            }
            for (int w = 0; w < 3; ++w) {
                const int kind = (int)rnd(4);
                int off[4];
                for (int k = 0; k < 4; ++k) off[k] = (int)rnd(15) - 7;
                if (kind == 1) sao[(size_t)c * 4 + w] = sao_pack(1, 0, (int)rnd(32), off);
                if (kind == 2) sao[(size_t)c * 4 + w] = sao_pack(2, (int)rnd(4), 0, off);
                if (kind == 3 && c > 0) sao[(size_t)c * 4 + w] = sao[(size_t)(c - 1) * 4 + w];  // merge candidates
            }
        }
        const bool use_sao = rnd(2) != 0;
        const PicSyn ps{cus.data(), coef.data(), qpp.data(), use_sao ? sao.data() : nullptr, mb_w, mb_h,
                        rnd(2) ? 3 : 0, 1};
        const uint32_t cap = (uint32_t)(end - first) * 16384 + 1024;
        std::vector<uint8_t> a(cap), b(cap);
        std::vector<uint16_t> tok(kMaxCuTokens);
        uint8_t ctx[C_NUM];
        const uint32_t na = code_slice(a.data(), cap, islice, qp, ps, first, end, ctx, tok.data(), true);
        const uint32_t nb = code_slice(b.data(), cap, islice, qp, ps, first, end, ctx, tok.data(), false);
        if (na != nb || std::memcmp(a.data(), b.data(), na) != 0)
            throw std::runtime_error("hevc token path differs from direct coding (slice " + std::to_string(sl) + ")");
    }
    return slices;
}

}  // namespace hevc
}  // namespace mx
