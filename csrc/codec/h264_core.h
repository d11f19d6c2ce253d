// H.264 Constrained-Baseline building blocks shared by the HIP encoder kernels
// (h264_kernels.hip) and the CPU encoder (h264_cpu.cpp): bit writer, 4x4 integer
// transforms, (de)quantisation, CAVLC residual block coding, and parameter-set /
// slice-header syntax.  Every function is __host__ __device__ and works on values in
// registers, so the GPU kernels decide the data layout and parallel decomposition.
//
// Replaces the fixed-function NVENC encoder behind `nvh264enc` (reference Dockerfile:210)
// and the x264 software fallback (README.md:21) -- see SURVEY.md C35/C36/C43.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h264_tables.h"

#define MXHD __host__ __device__ __forceinline__

namespace mx {
namespace h264 {

// ---------------------------------------------------------------- bit writing
// MSB-first bit writer into 32-bit words (word 0 bit 31 = first bit).  `Counting`
// variant only accumulates the length, used to size headers before placement.
struct BitWriter {
    uint32_t* words;
    uint32_t nwords;
    uint64_t acc;
    int nacc;
    uint32_t bits;

    MXHD void init(uint32_t* w) {
        words = w;
        nwords = 0;
        acc = 0;
        nacc = 0;
        bits = 0;
    }
    // n in [0,32]
    MXHD void put(uint32_t v, int n) {
        if (n <= 0) return;
        uint64_t m = (n == 32) ? 0xffffffffull : ((1ull << n) - 1);
        acc = (acc << n) | (v & m);
        nacc += n;
        bits += n;
        if (nacc >= 32) {
            words[nwords++] = (uint32_t)(acc >> (nacc - 32));
            nacc -= 32;
        }
    }
    MXHD void flush() {
        if (nacc > 0) {
            words[nwords++] = (uint32_t)(acc << (32 - nacc));
            nacc = 0;
            acc = 0;
        }
    }
};

struct BitCounter {
    uint32_t bits;
    MXHD void init(uint32_t*) { bits = 0; }
    MXHD void put(uint32_t, int n) { bits += (n > 0 ? n : 0); }
    MXHD void flush() {}
};

MXHD int ilog2_u32(uint32_t v) {  // floor(log2(v)), v > 0 (one v_ffbh on the GPU, not a shift loop)
    return 31 - __builtin_clz(v);
}

MXHD int ue_len(uint32_t k) { return 2 * ilog2_u32(k + 1) + 1; }
MXHD int se_len(int v) { return ue_len(v > 0 ? 2 * v - 1 : -2 * v); }

template <class W>
MXHD void put_ue(W& w, uint32_t k) {
    uint32_t v = k + 1;
    int nb = ilog2_u32(v);
    // nb leading zeros, then nb+1 bits of v
    if (nb > 0) w.put(0, nb);
    if (nb + 1 > 32) {
        w.put(v >> 16, nb + 1 - 16);
        w.put(v & 0xffff, 16);
    } else {
        w.put(v, nb + 1);
    }
}
template <class W>
MXHD void put_se(W& w, int v) {
    put_ue(w, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v));
}

// ---------------------------------------------------------------- transforms
// Forward core transform Y = Cf X Cf^T of a 4x4 residual block (raster order).
MXHD void fdct4x4(const int* x, int* y) {
    int t[16];
    for (int i = 0; i < 4; ++i) {  // rows
        int s03 = x[i * 4 + 0] + x[i * 4 + 3], d03 = x[i * 4 + 0] - x[i * 4 + 3];
        int s12 = x[i * 4 + 1] + x[i * 4 + 2], d12 = x[i * 4 + 1] - x[i * 4 + 2];
        t[i * 4 + 0] = s03 + s12;
        t[i * 4 + 1] = 2 * d03 + d12;
        t[i * 4 + 2] = s03 - s12;
        t[i * 4 + 3] = d03 - 2 * d12;
    }
    for (int j = 0; j < 4; ++j) {  // columns
        int s03 = t[0 * 4 + j] + t[3 * 4 + j], d03 = t[0 * 4 + j] - t[3 * 4 + j];
        int s12 = t[1 * 4 + j] + t[2 * 4 + j], d12 = t[1 * 4 + j] - t[2 * 4 + j];
        y[0 * 4 + j] = s03 + s12;
        y[1 * 4 + j] = 2 * d03 + d12;
        y[2 * 4 + j] = s03 - s12;
        y[3 * 4 + j] = d03 - 2 * d12;
    }
}

// Inverse core transform (8.5.12.2) of dequantised coefficients d, producing the
// residual r = (h + 32) >> 6.
MXHD void idct4x4(const int* d, int* r) {
    int f[16];
    for (int i = 0; i < 4; ++i) {
        int e0 = d[i * 4 + 0] + d[i * 4 + 2];
        int e1 = d[i * 4 + 0] - d[i * 4 + 2];
        int e2 = (d[i * 4 + 1] >> 1) - d[i * 4 + 3];
        int e3 = d[i * 4 + 1] + (d[i * 4 + 3] >> 1);
        f[i * 4 + 0] = e0 + e3;
        f[i * 4 + 1] = e1 + e2;
        f[i * 4 + 2] = e1 - e2;
        f[i * 4 + 3] = e0 - e3;
    }
    for (int j = 0; j < 4; ++j) {
        int g0 = f[0 * 4 + j] + f[2 * 4 + j];
        int g1 = f[0 * 4 + j] - f[2 * 4 + j];
        int g2 = (f[1 * 4 + j] >> 1) - f[3 * 4 + j];
        int g3 = f[1 * 4 + j] + (f[3 * 4 + j] >> 1);
        r[0 * 4 + j] = (g0 + g3 + 32) >> 6;
        r[1 * 4 + j] = (g1 + g2 + 32) >> 6;
        r[2 * 4 + j] = (g1 - g2 + 32) >> 6;
        r[3 * 4 + j] = (g0 - g3 + 32) >> 6;
    }
}

// 4x4 Hadamard (unnormalised) used for the Intra16x16 DC path (both directions).
MXHD void hadamard4x4(const int* x, int* y) {
    int t[16];
    for (int i = 0; i < 4; ++i) {
        int a = x[i * 4 + 0], b = x[i * 4 + 1], c = x[i * 4 + 2], d = x[i * 4 + 3];
        t[i * 4 + 0] = a + b + c + d;
        t[i * 4 + 1] = a + b - c - d;
        t[i * 4 + 2] = a - b - c + d;
        t[i * 4 + 3] = a - b + c - d;
    }
    for (int j = 0; j < 4; ++j) {
        int a = t[0 * 4 + j], b = t[1 * 4 + j], c = t[2 * 4 + j], d = t[3 * 4 + j];
        y[0 * 4 + j] = a + b + c + d;
        y[1 * 4 + j] = a + b - c - d;
        y[2 * 4 + j] = a - b - c + d;
        y[3 * 4 + j] = a - b + c - d;
    }
}

// ---------------------------------------------------------------- quantisation
MXHD int qclip(int v, int lim) { return v > lim ? lim : (v < -lim ? -lim : v); }

// Levels are clamped so every level stays codable with Baseline CAVLC escape codes.
constexpr int kMaxLevel = 2047;

// Quantise a transformed 4x4 block (raster). `start` = 1 skips the DC (AC-only blocks).
// Returns number of non-zero levels.
MXHD int quant4x4(const int* y, int* z, int qp, bool intra, int start) {
    const int qm = qp % 6, qbits = 15 + qp / 6;
    const int f = intra ? ((1 << qbits) / 3) : ((1 << qbits) / 6);
    int nz = 0;
    for (int i = 0; i < 16; ++i) {
        if (i < start) {
            z[i] = 0;
            continue;
        }
        int v = y[i];
        int a = v < 0 ? -v : v;
        int q = (int)(((int64_t)a * kQuantMF[qm][kPosClass[i]] + f) >> qbits);
        q = q > kMaxLevel ? kMaxLevel : q;
        z[i] = v < 0 ? -q : q;
        nz += (q != 0);
    }
    return nz;
}

// Dequantise (8.5.12.1, flat scaling lists): d = c * V << (qp/6).  DC left untouched
// when `start` = 1 (it comes from the separate DC path).
MXHD void dequant4x4(const int* z, int* d, int qp, int start) {
    const int qm = qp % 6, qs = qp / 6;
    for (int i = start; i < 16; ++i) d[i] = z[i] * kDequantV[qm][kPosClass[i]] * (1 << qs);  // multiply: << of negatives is UB
}

// Intra16x16 luma DC: forward Hadamard of the 16 DCs, /2 with rounding, quantise.
MXHD int quant_dc_luma(const int* dc_in, int* z, int qp) {
    int h[16];
    hadamard4x4(dc_in, h);
    const int qm = qp % 6, qbits = 16 + qp / 6;
    const int f = 2 * ((1 << (qbits - 1)) / 3);
    int nz = 0;
    for (int i = 0; i < 16; ++i) {
        int v = h[i] >> 1;
        int a = v < 0 ? -v : v;
        int q = (int)(((int64_t)a * kQuantMF[qm][0] + f) >> qbits);
        q = q > kMaxLevel ? kMaxLevel : q;
        z[i] = v < 0 ? -q : q;
        nz += (q != 0);
    }
    return nz;
}

// Inverse of the luma DC path (8.5.10): f = H c H, dcY = scaled f.  Output raster 4x4 of
// dequantised DC values for the 16 blocks (index = blkY*4 + blkX).
MXHD void dequant_dc_luma(const int* z, int* dcY, int qp) {
    int f[16];
    hadamard4x4(z, f);
    const int ls = 16 * kDequantV[qp % 6][0];
    const int qs = qp / 6;
    for (int i = 0; i < 16; ++i) {
        if (qp >= 36)
            dcY[i] = f[i] * ls * (1 << (qs - 6));
        else
            dcY[i] = (f[i] * ls + (1 << (5 - qs))) >> (6 - qs);
    }
}

// Chroma DC 2x2 (raster c0 c1 / c2 c3).
MXHD int quant_dc_chroma(const int* dc_in, int* z, int qpc, bool intra) {
    int a0 = dc_in[0] + dc_in[1], a1 = dc_in[0] - dc_in[1];
    int a2 = dc_in[2] + dc_in[3], a3 = dc_in[2] - dc_in[3];
    int h[4] = {a0 + a2, a1 + a3, a0 - a2, a1 - a3};
    const int qm = qpc % 6, qbits = 16 + qpc / 6;
    const int f = intra ? 2 * ((1 << (qbits - 1)) / 3) : 2 * ((1 << (qbits - 1)) / 6);
    int nz = 0;
    for (int i = 0; i < 4; ++i) {
        int v = h[i];
        int a = v < 0 ? -v : v;
        int q = (int)(((int64_t)a * kQuantMF[qm][0] + f) >> qbits);
        q = q > kMaxLevel ? kMaxLevel : q;
        z[i] = v < 0 ? -q : q;
        nz += (q != 0);
    }
    return nz;
}

MXHD void dequant_dc_chroma(const int* z, int* dcC, int qpc) {
    int a0 = z[0] + z[1], a1 = z[0] - z[1];
    int a2 = z[2] + z[3], a3 = z[2] - z[3];
    int f[4] = {a0 + a2, a1 + a3, a0 - a2, a1 - a3};
    const int ls = 16 * kDequantV[qpc % 6][0];
    for (int i = 0; i < 4; ++i) dcC[i] = (f[i] * ls * (1 << (qpc / 6))) >> 5;
}

MXHD int chroma_qp(int qp, int offset) {
    int q = qp + offset;
    q = q < 0 ? 0 : (q > 51 ? 51 : q);
    return kChromaQp[q];
}

// ---------------------------------------------------------------- CAVLC
MXHD int nc_table(int nC) {
    if (nC < 0) return 4;
    if (nC < 2) return 0;
    if (nC < 4) return 1;
    if (nC < 8) return 2;
    return 3;
}

// Code one residual block with CAVLC (9.2).  `coef` holds maxNum levels in scan order.
// Returns TotalCoeff.
template <class W>
MXHD int cavlc_block(W& w, const int16_t* coef, int maxNum, int nC) {
    // Streaming form (no per-block level/run arrays: on the GPU those would be dynamically
    // indexed private arrays, i.e. scratch memory).  Three passes over coef[], highest
    // frequency first.
    int total = 0, last = -1, t1 = 0;
    bool t1_open = true;
    for (int i = maxNum - 1; i >= 0; --i) {
        const int c = coef[i];
        if (c != 0) {
            if (last < 0) last = i;
            if (t1_open) {
                if ((c == 1 || c == -1) && t1 < 3) ++t1;
                else t1_open = false;
            }
            ++total;
        }
    }
    const int tab = nc_table(nC);
    if (total == 0) {
        w.put(kCoeffToken0[tab].code, kCoeffToken0[tab].len);
        return 0;
    }
    const Vlc ct = kCoeffToken[tab][total - 1][t1];
    w.put(ct.code, ct.len);
    // trailing-one signs, then levels
    int sl = (total > 10 && t1 < 3) ? 1 : 0;
    int k = 0;
    for (int i = last; i >= 0; --i) {
        const int l = coef[i];
        if (l == 0) continue;
        if (k < t1) {
            w.put(l < 0 ? 1u : 0u, 1);
            ++k;
            continue;
        }
        int code = l > 0 ? 2 * l - 2 : -2 * l - 1;
        if (k == t1 && t1 < 3) code -= 2;
        if (sl == 0) {
            if (code < 14) {
                w.put(1, code + 1);
            } else if (code < 30) {
                w.put(1, 15);  // prefix 14
                w.put(code - 14, 4);
            } else {
                w.put(1, 16);  // prefix 15
                w.put(code - 30, 12);
            }
        } else {
            if (code < (15 << sl)) {
                w.put(1, (code >> sl) + 1);
                w.put(code & ((1 << sl) - 1), sl);
            } else {
                w.put(1, 16);
                w.put(code - (15 << sl), 12);
            }
        }
        if (sl == 0) sl = 1;
        const int a = l < 0 ? -l : l;
        if (a > (3 << (sl - 1)) && sl < 6) ++sl;
        ++k;
    }
    const int total_zeros = last + 1 - total;
    if (total < maxNum) {
        const Vlc tz = (maxNum == 4) ? kTotalZerosDc[total - 1][total_zeros] : kTotalZeros[total - 1][total_zeros];
        w.put(tz.code, tz.len);
    }
    // run_before: zeros directly below each non-zero (highest first), except the lowest one
    int zl = total_zeros;
    int i = last;
    for (int seen = 0; seen < total - 1 && zl > 0; ++seen) {
        int j = i - 1, rb = 0;
        while (coef[j] == 0) {
            ++rb;
            --j;
        }
        const Vlc v = kRunBefore[(zl > 7 ? 7 : zl) - 1][rb];
        w.put(v.code, v.len);
        zl -= rb;
        i = j;
    }
    return total;
}

// ---------------------------------------------------------------- syntax structures
struct SeqParams {
    int width, height;      // display size (luma samples)
    int mb_w, mb_h;         // coded size in macroblocks
    int level_idc;          // e.g. 42
    int log2_max_frame_num; // 4..16
    int fps_num, fps_den;   // VUI timing
};

// Choose the lowest level that fits the coded size and rate (Table A-1 subset).
MXHD int pick_level(int mbs, int fps) {
    long mbps = (long)mbs * fps;
    if (mbs <= 1620 && mbps <= 40500) return 30;
    if (mbs <= 3600 && mbps <= 108000) return 31;
    if (mbs <= 5120 && mbps <= 216000) return 32;
    if (mbs <= 8192 && mbps <= 245760) return 40;
    if (mbs <= 8704 && mbps <= 522240) return 42;
    if (mbs <= 22080 && mbps <= 589824) return 50;
    if (mbs <= 36864 && mbps <= 983040) return 51;
    if (mbs <= 36864) return 52;
    if (mbs <= 139264 && mbps <= 4177920) return 60;
    if (mbs <= 139264 && mbps <= 8355840) return 61;
    return 62;
}

// seq_parameter_set_rbsp (7.3.2.1.1), Constrained Baseline, POC type 2, with VUI timing.
template <class W>
MXHD void write_sps(W& w, const SeqParams& p) {
    w.put(66, 8);        // profile_idc: Baseline
    w.put(0xC0, 8);      // constraint_set0_flag=1, constraint_set1_flag=1 (Constrained Baseline)
    w.put(p.level_idc, 8);
    put_ue(w, 0);        // seq_parameter_set_id
    put_ue(w, p.log2_max_frame_num - 4);
    put_ue(w, 2);        // pic_order_cnt_type = 2 (output order == decode order)
    put_ue(w, 1);        // max_num_ref_frames
    w.put(0, 1);         // gaps_in_frame_num_value_allowed_flag
    put_ue(w, p.mb_w - 1);
    put_ue(w, p.mb_h - 1);
    w.put(1, 1);         // frame_mbs_only_flag
    w.put(1, 1);         // direct_8x8_inference_flag
    const int crop_r = (p.mb_w * 16 - p.width) / 2, crop_b = (p.mb_h * 16 - p.height) / 2;
    if (crop_r || crop_b) {
        w.put(1, 1);
        put_ue(w, 0);
        put_ue(w, crop_r);
        put_ue(w, 0);
        put_ue(w, crop_b);
    } else {
        w.put(0, 1);
    }
    w.put(1, 1);         // vui_parameters_present_flag
    w.put(0, 1);         // aspect_ratio_info_present_flag
    w.put(0, 1);         // overscan_info_present_flag
    w.put(1, 1);         // video_signal_type_present_flag
    w.put(5, 3);         //   video_format: unspecified
    w.put(0, 1);         //   video_full_range_flag: limited (BT.709 studio swing)
    w.put(1, 1);         //   colour_description_present_flag
    w.put(1, 8);         //   colour_primaries BT.709
    w.put(1, 8);         //   transfer_characteristics BT.709
    w.put(1, 8);         //   matrix_coefficients BT.709
    w.put(0, 1);         // chroma_loc_info_present_flag
    w.put(1, 1);         // timing_info_present_flag
    w.put((uint32_t)p.fps_den, 32);      // num_units_in_tick
    w.put((uint32_t)(2 * p.fps_num), 32);  // time_scale
    w.put(0, 1);         // fixed_frame_rate_flag (variable: frames are paced by the app)
    w.put(0, 1);         // nal_hrd_parameters_present_flag
    w.put(0, 1);         // vcl_hrd_parameters_present_flag
    w.put(0, 1);         // pic_struct_present_flag
    w.put(1, 1);         // bitstream_restriction_flag
    w.put(1, 1);         //   motion_vectors_over_pic_boundaries_flag
    put_ue(w, 0);        //   max_bytes_per_pic_denom (no limit)
    put_ue(w, 0);        //   max_bits_per_mb_denom
    put_ue(w, 16);       //   log2_max_mv_length_horizontal
    put_ue(w, 16);       //   log2_max_mv_length_vertical
    put_ue(w, 0);        //   max_num_reorder_frames (no reordering: low latency)
    put_ue(w, 1);        //   max_dec_frame_buffering
    w.put(1, 1);         // rbsp_stop_one_bit
    w.flush();
}

// pic_parameter_set_rbsp (7.3.2.2)
template <class W>
MXHD void write_pps(W& w, int init_qp, int chroma_qp_offset) {
    put_ue(w, 0);  // pic_parameter_set_id
    put_ue(w, 0);  // seq_parameter_set_id
    w.put(0, 1);   // entropy_coding_mode_flag: CAVLC
    w.put(0, 1);   // bottom_field_pic_order_in_frame_present_flag
    put_ue(w, 0);  // num_slice_groups_minus1
    put_ue(w, 0);  // num_ref_idx_l0_default_active_minus1
    put_ue(w, 0);  // num_ref_idx_l1_default_active_minus1
    w.put(0, 1);   // weighted_pred_flag
    w.put(0, 2);   // weighted_bipred_idc
    put_se(w, init_qp - 26);
    put_se(w, 0);  // pic_init_qs_minus26
    put_se(w, chroma_qp_offset);
    w.put(1, 1);   // deblocking_filter_control_present_flag
    w.put(0, 1);   // constrained_intra_pred_flag
    w.put(0, 1);   // redundant_pic_cnt_present_flag
    w.put(1, 1);   // rbsp_stop_one_bit
    w.flush();
}

struct SliceParams {
    int first_mb;
    int idr;          // 1 = IDR picture (I slice), 0 = P
    int frame_num;
    int log2_max_frame_num;
    int idr_pic_id;
    int qp_delta;     // slice_qp_delta relative to pic_init_qp
    int disable_deblock;  // disable_deblocking_filter_idc
};

// slice_header (7.3.3) for our subset: single PPS, POC type 2, one reference, no
// reordering, sliding-window marking.
template <class W>
MXHD void write_slice_header(W& w, const SliceParams& s) {
    put_ue(w, (uint32_t)s.first_mb);
    put_ue(w, s.idr ? 7u : 5u);  // slice_type: I (7) / P (5), "all slices same type"
    put_ue(w, 0);                // pic_parameter_set_id
    w.put((uint32_t)s.frame_num, s.log2_max_frame_num);
    if (s.idr) put_ue(w, (uint32_t)s.idr_pic_id);
    if (!s.idr) {
        w.put(0, 1);  // num_ref_idx_active_override_flag
        w.put(0, 1);  // ref_pic_list_modification_flag_l0
    }
    // dec_ref_pic_marking (nal_ref_idc != 0)
    if (s.idr) {
        w.put(0, 1);  // no_output_of_prior_pics_flag
        w.put(0, 1);  // long_term_reference_flag
    } else {
        w.put(0, 1);  // adaptive_ref_pic_marking_mode_flag
    }
    put_se(w, s.qp_delta);
    put_ue(w, (uint32_t)s.disable_deblock);
    if (s.disable_deblock != 1) {
        put_se(w, 0);  // slice_alpha_c0_offset_div2
        put_se(w, 0);  // slice_beta_offset_div2
    }
}

// ---------------------------------------------------------------- motion vectors
struct Mv {
    int x, y;
};
MXHD int median3(int a, int b, int c) {
    int mx = a > b ? a : b;
    int mn = a < b ? a : b;
    return c > mx ? mx : (c < mn ? mn : c);
}

// Neighbour (A left, B top, C top-right or D top-left) for 16x16 mv prediction.
struct MvNb {
    bool avail;  // neighbour MB exists (inside picture and slice)
    int ref;     // -1 intra/unavailable, 0 = L0 ref 0
    Mv mv;
};

// 8.4.1.3 median luma mv prediction for a 16x16 partition, refIdx 0.
MXHD Mv predict_mv16x16(MvNb a, MvNb b, MvNb c) {
    if (!a.avail) { a.ref = -1; a.mv = {0, 0}; }
    if (!b.avail) { b.ref = -1; b.mv = {0, 0}; }
    if (!c.avail) { c.ref = -1; c.mv = {0, 0}; }
    if (!b.avail && !c.avail && a.avail) {
        b = a;
        c = a;
    }
    int n = (a.ref == 0) + (b.ref == 0) + (c.ref == 0);
    if (n == 1) {
        if (a.ref == 0) return a.mv;
        if (b.ref == 0) return b.mv;
        return c.mv;
    }
    return Mv{median3(a.mv.x, b.mv.x, c.mv.x), median3(a.mv.y, b.mv.y, c.mv.y)};
}

// 8.4.1.1 P_Skip motion vector.
MXHD Mv predict_mv_skip(MvNb a, MvNb b, MvNb c) {
    if (!a.avail || !b.avail) return Mv{0, 0};
    if (a.ref == 0 && a.mv.x == 0 && a.mv.y == 0) return Mv{0, 0};
    if (b.ref == 0 && b.mv.x == 0 && b.mv.y == 0) return Mv{0, 0};
    return predict_mv16x16(a, b, c);
}

// cbp (bits 0..3 luma 8x8, bits 4..5 chroma) -> codeNum for me(v)
MXHD int cbp_to_codenum(int cbp, bool intra) {
    const uint8_t* t = intra ? kCodeNumToCbpIntra : kCodeNumToCbpInter;
    for (int i = 0; i < 48; ++i)
        if (t[i] == cbp) return i;
    return 0;
}

MXHD int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// ---------------------------------------------------------------- interpolation
// Reference sample fetch with picture-edge clamping (8.4.2.2.1 eq. 8-228/8-229).
MXHD int ref_px(const uint8_t* p, int pitch, int w, int h, int x, int y) {
    x = x < 0 ? 0 : (x >= w ? w - 1 : x);
    y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    return p[y * pitch + x];
}

MXHD int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

// Horizontal half-sample intermediate b1 at (x+1/2, y).
MXHD int half_h1(const uint8_t* p, int pitch, int w, int h, int x, int y) {
    return tap6(ref_px(p, pitch, w, h, x - 2, y), ref_px(p, pitch, w, h, x - 1, y), ref_px(p, pitch, w, h, x, y),
                ref_px(p, pitch, w, h, x + 1, y), ref_px(p, pitch, w, h, x + 2, y), ref_px(p, pitch, w, h, x + 3, y));
}
// Vertical half-sample intermediate h1 at (x, y+1/2).
MXHD int half_v1(const uint8_t* p, int pitch, int w, int h, int x, int y) {
    return tap6(ref_px(p, pitch, w, h, x, y - 2), ref_px(p, pitch, w, h, x, y - 1), ref_px(p, pitch, w, h, x, y),
                ref_px(p, pitch, w, h, x, y + 1), ref_px(p, pitch, w, h, x, y + 2), ref_px(p, pitch, w, h, x, y + 3));
}

// Luma sample at quarter-sample position (x4, y4) (8.4.2.2.1, Table 8-12).
MXHD int luma_qpel(const uint8_t* p, int pitch, int w, int h, int x4, int y4) {
    const int xi = x4 >> 2, yi = y4 >> 2, xf = x4 & 3, yf = y4 & 3;
    const int G = ref_px(p, pitch, w, h, xi, yi);
    if ((xf | yf) == 0) return G;
    auto b_at = [&](int yy) { return clip255((half_h1(p, pitch, w, h, xi, yy) + 16) >> 5); };
    auto h_at = [&](int xx) { return clip255((half_v1(p, pitch, w, h, xx, yi) + 16) >> 5); };
    auto j_val = [&]() {
        int j1 = tap6(half_h1(p, pitch, w, h, xi, yi - 2), half_h1(p, pitch, w, h, xi, yi - 1),
                      half_h1(p, pitch, w, h, xi, yi), half_h1(p, pitch, w, h, xi, yi + 1),
                      half_h1(p, pitch, w, h, xi, yi + 2), half_h1(p, pitch, w, h, xi, yi + 3));
        return clip255((j1 + 512) >> 10);
    };
    if (yf == 0) {
        const int b = b_at(yi);
        if (xf == 2) return b;
        const int other = (xf == 1) ? G : ref_px(p, pitch, w, h, xi + 1, yi);
        return (other + b + 1) >> 1;  // a / c
    }
    if (xf == 0) {
        const int hh = h_at(xi);
        if (yf == 2) return hh;
        const int other = (yf == 1) ? G : ref_px(p, pitch, w, h, xi, yi + 1);
        return (other + hh + 1) >> 1;  // d / n
    }
    if (xf == 2 && yf == 2) return j_val();
    if (xf == 2) {  // f (yf=1) / q (yf=3)
        const int bb = (yf == 1) ? b_at(yi) : b_at(yi + 1);
        return (bb + j_val() + 1) >> 1;
    }
    if (yf == 2) {  // i (xf=1) / k (xf=3)
        const int hh = (xf == 1) ? h_at(xi) : h_at(xi + 1);
        return (hh + j_val() + 1) >> 1;
    }
    // diagonal quarter positions e, g, p, r: average of the nearest b/s and h/m
    const int bb = (yf == 1) ? b_at(yi) : b_at(yi + 1);
    const int hh = (xf == 1) ? h_at(xi) : h_at(xi + 1);
    return (bb + hh + 1) >> 1;
}

// Chroma sample (component comp of interleaved NV12 UV plane) at 1/8-sample position.
MXHD int chroma_pred8(const uint8_t* uv, int pitch, int cw, int ch, int comp, int x8, int y8) {
    const int xi = x8 >> 3, yi = y8 >> 3, xf = x8 & 7, yf = y8 & 7;
    auto g = [&](int x, int y) {
        x = x < 0 ? 0 : (x >= cw ? cw - 1 : x);
        y = y < 0 ? 0 : (y >= ch ? ch - 1 : y);
        return (int)uv[y * pitch + 2 * x + comp];
    };
    if ((xf | yf) == 0) return g(xi, yi);  // full-sample vector: the weights are 64, 0, 0, 0
    const int A = g(xi, yi), B = g(xi + 1, yi), C = g(xi, yi + 1), D = g(xi + 1, yi + 1);
    return ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
}

// Rough Lagrange multiplier for SAD-domain motion/mode decisions.
MXHD int lambda_sad(int qp) {
    constexpr uint8_t tab[52] = {1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,
                                 2,  2,  2,  2,  3,  3,  3,  4,  4,  4,  5,  6,  6,  7,  8,  9,  10, 11,
                                 13, 14, 16, 18, 20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72};
    return tab[qp < 0 ? 0 : (qp > 51 ? 51 : qp)];
}

// Approximate bits of an mvd component in quarter-pel units.
MXHD int mvd_bits(int d) { return se_len(d); }

}  // namespace h264
}  // namespace mx
