// HIP/CDNA4 kernels of the HEVC encoder (BASELINE.json "4K60 HEVC").
//
// Decomposition (gfx950: 256 CUs, wave64):
//  * k_hevc_inter  one wave per 16x16 CU (4 per workgroup) after the shared H.264 motion
//                  search (k_hpel + k_me_full): 8-tap luma / 4-tap chroma motion
//                  compensation, the 16x16 / 8x8 core transforms as LDS-staged
//                  matrix products (4 luma + 2 chroma outputs per lane per stage),
//                  quantisation, normative inverse transform and reconstruction, coded
//                  sub-block / last-position summaries by wave reductions.
//  * k_hevc_intra  one workgroup per slice, one wave per unit row; the rows of a slice run
//                  as a wavefront (a unit waits until the row above finished the units
//                  above and above-right: per-row progress counters in LDS, no workgroup
//                  barriers) with the left column and the bottom rows exchanged through LDS.
//  * k_hevc_bins / k_hevc_tokscan / k_hevc_tokgather / k_hevc_arith  CABAC in two phases:
//                  every CTU binarised at once (one wave per CTU, one lane per syntax part,
//                  hevc_core.h binarise_part) into bin tokens laid out densely in decoding order, then
//                  one wave per slice runs its token run through the arithmetic coder.
//  * k_hevc_layout / k_hevc_decide  slice layout (rows for I, cost-balanced raster runs for
//                  P) and the per-slice skip / merge / AMVP decisions.
//  * k_hevc_qpy + k_hevc_deblock + k_hevc_sse  in-loop deblocking (QP chain per slice, one
//                  thread per 4-sample CU-edge segment, vertical then horizontal pass) and the
//                  distortion of the final picture.
//  * k_hevc_pack   one workgroup per slice copies the slice bytes (16-byte stores) into
//                  pinned host memory at 16-byte aligned offsets; workgroup 0 writes the
//                  header (lengths, overflow, distortion totals).
#include <hip/hip_runtime.h>

#include <algorithm>

#include <stdexcept>

#include "h264_core.h"
#include "h264_gpu.h"
#include "h264_mb.h"
#include "hevc_core.h"
#include "hevc_encoder.h"

namespace mx {
namespace hevc {

namespace {

// Cross-row exchanges without LDS (CDNA4 v_permlane16/32_swap with both operands = v): the
// swapped pair holds {v, v ^ 16} (resp. {v, v ^ 32}) in some order on every lane, so their
// sum / max / or is the xor-16 (xor-32) step of a butterfly -- no ds_bpermute round trip.
__device__ __forceinline__ void xrow16(uint32_t v, uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    a = r[0];
    b = r[1];
}
__device__ __forceinline__ void xrow32(uint32_t v, uint32_t& a, uint32_t& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    a = r[0];
    b = r[1];
}
// Wave sum, every lane gets it (called with the whole wave active): quad and row-of-16 sums
// with DPP (quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, row_ror 8), then the four rows with the
// two permlane swaps -- all VALU, no LDS latency on the (often serial) reduction chains.
__device__ __forceinline__ int wsum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
    uint32_t a, b;
    xrow16((uint32_t)v, a, b);
    v = (int)(a + b);
    xrow32((uint32_t)v, a, b);
    return (int)(a + b);
}
// reductions inside aligned groups of G lanes (G = 8 or 16): every lane gets its group's value
template <int G>
__device__ __forceinline__ int gsum(int v) {
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int G>
__device__ __forceinline__ int gmax(int v) {
    for (int o = G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
// wave max / or: the same DPP + permlane butterfly as wsum
__device__ __forceinline__ int wmax(int v) {
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false));
    uint32_t a, b;
    xrow16((uint32_t)v, a, b);
    v = max((int)a, (int)b);
    xrow32((uint32_t)v, a, b);
    return max((int)a, (int)b);
}
__device__ __forceinline__ uint32_t wor(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
    uint32_t a, b;
    xrow16(v, a, b);
    xrow32(a | b, a, b);
    return a | b;
}

// LDS hand-off between the lanes of ONE wave (its own LDS writes visible to its own later reads;
// LDS operations of a wave complete in order): no workgroup barrier, so the waves of a workgroup
// may take different branches around it.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Stage separator of the TU helpers: wave-local (every wave has its own LDS scratch; the intra
// wavefront's rows synchronise through progress counters, not workgroup barriers).
template <bool kWaveLocal>
__device__ __forceinline__ void tu_sync() {
    wave_lds_sync();  // both users run their waves alone (the intra wavefront through progress counters)
}

// Transform matrices in LDS (filled once per workgroup).
struct alignas(16) Mats {
    int16_t t16[256];
    int16_t t8[64];
    int16_t t4[16];
    int16_t tt16[256];  // transposed: tt16[y * 16 + k] = t16[k * 16 + y] (inverse stages)
    int16_t tt8[64];
    int16_t tt4[16];
};
__device__ __forceinline__ void fill_mats(Mats& m) {
    for (int i = threadIdx.x; i < 256 + 64 + 16; i += blockDim.x) {
        if (i < 256) {
            m.t16[i] = (int16_t)dct_coef(4, i >> 4, i & 15);
            m.tt16[i] = (int16_t)dct_coef(4, i & 15, i >> 4);
        } else if (i < 320) {
            m.t8[i - 256] = (int16_t)dct_coef(3, (i - 256) >> 3, (i - 256) & 7);
            m.tt8[i - 256] = (int16_t)dct_coef(3, (i - 256) & 7, (i - 256) >> 3);
        } else {
            m.t4[i - 320] = (int16_t)dct_coef(2, (i - 320) >> 2, (i - 320) & 3);
            m.tt4[i - 320] = (int16_t)dct_coef(2, (i - 320) & 3, (i - 320) >> 2);
        }
    }
}

// Integer dot products of 16 / 8 int16 pairs from 16-byte aligned LDS rows with v_dot2 (two
// multiply-adds per VALU instruction, one ds_read_b128 per 8 values).  Exact: int32 sums.
typedef short mx_short2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2acc(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(mx_short2, a), __builtin_bit_cast(mx_short2, b), c, false);
}
__device__ __forceinline__ int dot8(const int16_t* a, const int16_t* b) {
    const uint4 x = *reinterpret_cast<const uint4*>(a), y = *reinterpret_cast<const uint4*>(b);
    return dot2acc(x.w, y.w, dot2acc(x.z, y.z, dot2acc(x.y, y.y, dot2acc(x.x, y.x, 0))));
}
__device__ __forceinline__ int dot4(const int16_t* a, const int16_t* b) {  // 8-byte aligned rows
    const uint2 x = *reinterpret_cast<const uint2*>(a), y = *reinterpret_cast<const uint2*>(b);
    return dot2acc(x.y, y.y, dot2acc(x.x, y.x, 0));
}
__device__ __forceinline__ int dot16(const int16_t* a, const int16_t* b) { return dot8(a, b) + dot8(a + 8, b + 8); }

// Per-wave TU scratch: residual / prediction / two int32 stage buffers for 256 luma +
// 2 x 64 chroma samples (code_tus keeps int16 stage values in them, laid out so that every
// transform stage reads contiguous 16-byte rows: see its comments).
struct alignas(16) TuBuf {
    int16_t res[384];
    uint8_t pred[384];
    int32_t a[384];
    int32_t b[384];
};

// One wave transforms, quantises and reconstructs its CU's three TUs.  Lane mapping per
// stage: luma outputs lane*4 .. lane*4+3, chroma outputs (lane&31)*2 .. +1 of component
// lane>>5.  tu_sync<kInterCu>() (wave-local) separates the stages; intra CUs (kInterCu false)
// keep their reconstruction in t.pred for the neighbours, inter CUs leave t.pred (the prediction)
// intact for the split tree after it.
struct TuResult {
    int last[3];
    uint32_t csbf[3];
    int nz[3];
    int sse[3];     // over the display area (PSNR)
    int sse_full;   // over the whole CU (transform-tree decision, as the CPU encoder)
    int sse_y_full; // luma only, whole CU (residual drop)
    uint32_t bits;  // cu_bits_est of the levels (unsplit tree)
    uint32_t bits_y;  // tu_bits_est of the luma TU
};

template <bool kInterCu>
__device__ __forceinline__ TuResult code_tus(TuBuf& t, const Mats& M, int qp, int qpc, bool intra, bool valid,
                                             int16_t* coef, uint8_t* rec_y, int pitch_y, uint8_t* rec_uv, int x0,
                                             int y0, int disp_w, int disp_h) {
    const int lane = threadIdx.x & 63;
    const int comp = lane >> 5, cl = lane & 31;
    // int16 views of the stage buffers: aT = forward stage 1 transposed (aT[k][y]), bT = the
    // dequantised levels transposed (bT[x][k]), a16 = inverse stage 1 (a16[y][x]); forward
    // stage 1 fits 16 bits (|res| <= 255, row sums of |T| <= 1024 before the >> 3 / >> 2)
    int16_t* aT = reinterpret_cast<int16_t*>(t.a);
    int16_t* a16 = reinterpret_cast<int16_t*>(t.a);
    int16_t* bT = reinterpret_cast<int16_t*>(t.b);
    // ---- forward stage 1 (rows): a[y][k] = sum_n T[k][n] res[y][n]
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = lane * 4 + j, y = idx >> 4, k = idx & 15;
            const int s = dot16(M.t16 + k * 16, t.res + y * 16);
            aT[k * 16 + y] = (int16_t)((s + 4) >> 3);
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = cl * 2 + j, y = idx >> 3, k = idx & 7;
            const int16_t* r = t.res + 256 + comp * 64;
            const int s = dot8(M.t8 + k * 8, r + y * 8);
            aT[256 + comp * 64 + k * 8 + y] = (int16_t)((s + 2) >> 2);
        }
    }
    tu_sync<kInterCu>();
    TuResult out;
    int lastl = -1, lastc = -1, nzl = 0, nzc = 0;
    uint32_t csl = 0, csc = 0;
    // ---- forward stage 2 (columns) + quantisation (levels kept in registers)
    int ll[4] = {0, 0, 0, 0}, lc[2] = {0, 0};
    int mxl = 0, mxc = 0;
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = lane * 4 + j, k2 = idx >> 4, k = idx & 15;
            const int s = dot16(M.t16 + k2 * 16, aT + k * 16);
            ll[j] = quant_coef((s + 512) >> 10, qp, 4, intra);
            nzl += ll[j] != 0;
            mxl = max(mxl, abs(ll[j]));
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = cl * 2 + j, k2 = idx >> 3, k = idx & 7;
            const int s = dot8(M.t8 + k2 * 8, aT + 256 + comp * 64 + k * 8);
            lc[j] = quant_coef((s + 256) >> 9, qpc, 3, intra);
            nzc += lc[j] != 0;
            mxc = max(mxc, abs(lc[j]));
        }
    }
    // decimation (wave-uniform decisions per TU), then levels / dequantised values / summaries
    const bool drop_y = tu_decimate(4, intra, wsum(nzl), wmax(mxl));
    const bool drop_cb = tu_decimate(3, intra, wsum(comp == 0 ? nzc : 0), wmax(comp == 0 ? mxc : 0));
    const bool drop_cr = tu_decimate(3, intra, wsum(comp == 1 ? nzc : 0), wmax(comp == 1 ? mxc : 0));
    const bool drop_c = comp ? drop_cr : drop_cb;
    if (drop_y)
        for (int j = 0; j < 4; ++j) ll[j] = 0;
    if (drop_c)
        for (int j = 0; j < 2; ++j) lc[j] = 0;
    if (!intra) {
        // trailing isolated +-1 trim (tu_encode rule), one TU after the other; the lane owning
        // the last level clears it
        for (int it = 0; it < kTrimIters; ++it) {
            int last = -1;
            for (int j = 0; j < 4; ++j)
                if (ll[j]) last = max(last, scan_index(4, (lane * 4 + j) & 15, (lane * 4 + j) >> 4));
            last = wmax(last);
            if (last < 0) break;
            int prev = -1, lv = 0;
            for (int j = 0; j < 4; ++j) {
                const int si = scan_index(4, (lane * 4 + j) & 15, (lane * 4 + j) >> 4);
                if (ll[j] && si < last) prev = max(prev, si);
                if (si == last) lv = abs(ll[j]);
            }
            prev = wmax(prev);
            lv = wmax(lv);
            if (lv != 1 || last - prev <= kTrimGap) break;
            for (int j = 0; j < 4; ++j)
                if (scan_index(4, (lane * 4 + j) & 15, (lane * 4 + j) >> 4) == last) ll[j] = 0;
        }
        for (int cc = 0; cc < 2; ++cc) {
            for (int it = 0; it < kTrimIters; ++it) {
                int last = -1;
                for (int j = 0; j < 2; ++j) {
                    const int idx = cl * 2 + j;
                    if (comp == cc && lc[j]) last = max(last, scan_index(3, idx & 7, idx >> 3));
                }
                last = wmax(last);
                if (last < 0) break;
                int prev = -1, lv = 0;
                for (int j = 0; j < 2; ++j) {
                    const int idx = cl * 2 + j, si = scan_index(3, idx & 7, idx >> 3);
                    if (comp == cc && lc[j] && si < last) prev = max(prev, si);
                    if (comp == cc && si == last) lv = abs(lc[j]);
                }
                prev = wmax(prev);
                lv = wmax(lv);
                if (lv != 1 || last - prev <= kTrimGap) break;
                for (int j = 0; j < 2; ++j) {
                    const int idx = cl * 2 + j;
                    if (comp == cc && scan_index(3, idx & 7, idx >> 3) == last) lc[j] = 0;
                }
            }
        }
    }
    nzl = nzc = 0;
    int lbits = 0, cbits = 0;  // tu_bits_est terms of this lane's levels
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = lane * 4 + j, k2 = idx >> 4, k = idx & 15;
            const int l = ll[j];
            if (l) lbits += 4 + 2 * (31 - __builtin_clz((uint32_t)abs(l)));
            const int si = scan_index(4, k, k2);
            coef[si] = (int16_t)l;
            bT[k * 16 + k2] = (int16_t)dequant_coef(l, qp, 4);
            if (l) {
                ++nzl;
                lastl = si > lastl ? si : lastl;
                csl |= 1u << (si >> 4);
            }
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = cl * 2 + j, k2 = idx >> 3, k = idx & 7;
            const int l = lc[j];
            if (l) cbits += 4 + 2 * (31 - __builtin_clz((uint32_t)abs(l)));
            const int si = scan_index(3, k, k2);
            coef[256 + comp * 64 + si] = (int16_t)l;
            bT[256 + comp * 64 + k * 8 + k2] = (int16_t)dequant_coef(l, qpc, 3);
            if (l) {
                ++nzc;
                lastc = si > lastc ? si : lastc;
                csc |= 1u << (si >> 4);
            }
        }
    }
    out.nz[0] = wsum(nzl);
    out.last[0] = wmax(lastl);
    out.csbf[0] = wor(csl);
    {
        const int n_cb = wsum(comp == 0 ? nzc : 0), n_cr = wsum(comp == 1 ? nzc : 0);
        out.nz[1] = n_cb;
        out.nz[2] = n_cr;
        out.last[1] = wmax(comp == 0 ? lastc : -1);
        out.last[2] = wmax(comp == 1 ? lastc : -1);
        out.csbf[1] = wor(comp == 0 ? csc : 0u);
        out.csbf[2] = wor(comp == 1 ? csc : 0u);
    }
    {
        const int bl = wsum(lbits), bcb = wsum(comp == 0 ? cbits : 0), bcr = wsum(comp == 1 ? cbits : 0);
        out.bits = (uint32_t)((out.nz[0] ? bl + 4 : 1) + (out.nz[1] ? bcb + 4 : 1) + (out.nz[2] ? bcr + 4 : 1));
        out.bits_y = (uint32_t)(out.nz[0] ? bl + 4 : 1);
    }
    tu_sync<kInterCu>();
    // ---- inverse stage 1 (columns): a[y][x] = clip16((sum_k T[k][y] b[k][x] + 64) >> 7)
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = lane * 4 + j, y = idx >> 4, x = idx & 15;
            const int s = dot16(M.tt16 + y * 16, bT + x * 16);
            a16[idx] = (int16_t)clip16((s + 64) >> 7);
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = cl * 2 + j, y = idx >> 3, x = idx & 7;
            const int s = dot8(M.tt8 + y * 8, bT + 256 + comp * 64 + x * 8);
            a16[256 + comp * 64 + idx] = (int16_t)clip16((s + 64) >> 7);
        }
    }
    tu_sync<kInterCu>();
    // ---- inverse stage 2 (rows) + reconstruction
    int sy = 0, sc = 0, sf = 0, syf = 0;
    if (valid) {
        const int y = lane >> 2, xb = (lane & 3) * 4;
        uint32_t packed = 0;
        for (int j = 0; j < 4; ++j) {
            const int x = xb + j;
            const int s = dot16(M.tt16 + x * 16, a16 + y * 16);
            const int r = out.nz[0] ? (s + 2048) >> 12 : 0;
            const int p = t.pred[y * 16 + x];
            const int v = clip255(p + r);
            const int e = p + t.res[y * 16 + x] - v;
            sy += (x0 + x < disp_w && y0 + y < disp_h) ? e * e : 0;
            sf += e * e;
            syf += e * e;
            packed |= (uint32_t)v << (8 * j);
            if (!kInterCu) t.pred[y * 16 + x] = (uint8_t)v;  // intra: reconstruction stays readable in LDS
        }
        *reinterpret_cast<uint32_t*>(rec_y + (size_t)(y0 + y) * pitch_y + x0 + xb) = packed;
        const int nzcomp = comp ? out.nz[2] : out.nz[1];
        for (int j = 0; j < 2; ++j) {
            const int idx = cl * 2 + j, yy = idx >> 3, x = idx & 7;
            const int s = dot8(M.tt8 + x * 8, a16 + 256 + comp * 64 + yy * 8);
            const int r = nzcomp ? (s + 2048) >> 12 : 0;
            const int o = 256 + comp * 64 + idx;
            const int p = t.pred[o];
            const int v = clip255(p + r);
            const int e = p + t.res[o] - v;
            if (!kInterCu) t.pred[o] = (uint8_t)v;
            const int xc = x0 / 2 + x, yc = y0 / 2 + yy;
            sc += (2 * xc < disp_w && 2 * yc < disp_h) ? e * e : 0;
            sf += e * e;
            rec_uv[(size_t)yc * pitch_y + 2 * xc + comp] = (uint8_t)v;
        }
    }
    out.sse[0] = wsum(sy);
    out.sse[1] = wsum(comp == 0 ? sc : 0);
    out.sse[2] = wsum(comp == 1 ? sc : 0);
    out.sse_full = wsum(sf);
    out.sse_y_full = wsum(syf);
    return out;
}

// The split transform tree of an inter CU (split_encode / tu_encode_t of the CPU encoder,
// same integer stages), computed by the whole wave: luma TU k = lanes 16k..16k+15 with 4
// coefficients each, chroma TU (comp, k) = lanes 8(4comp+k).. with 2 each; decimation and
// the trailing trim per TU through segmented shuffle reductions.  Levels go to lv (CU
// layout), the reconstruction to rec (TuBuf layout); t.a / t.b are the stage buffers.
// cu_summarise (hevc_core.h) of a split transform tree, by the whole wave: one ballot per
// luma TU (lane = scan index) and one per chroma component (lane = 16 * TU + scan index) give
// the coded masks, the rest is scalar (lane 0 alone walking 384 LDS levels cost ~1,100 VALU).
struct SplitSummary {
    uint8_t cbf, cbf_y4, cbf_c4, last[3], csbf_c[2], tu4;
    uint16_t csbf_y, cbf_y16;
    __device__ void apply(CuInfo& c) const {
        c.cbf = cbf;
        c.cbf_y4 = cbf_y4;
        c.tu4 = tu4;
        c.cbf_y16 = cbf_y16;
        c.cbf_c4 = cbf_c4;
        c.last[0] = last[0];
        c.last[1] = last[1];
        c.last[2] = last[2];
        c.csbf_y = csbf_y;
        c.csbf_c[0] = csbf_c[0];
        c.csbf_c[1] = csbf_c[1];
    }
};
__device__ SplitSummary split_summary_wave(const int16_t* co, int lane, int tu4) {
    SplitSummary s = {};
    s.tu4 = (uint8_t)tu4;
    uint32_t lsum = 0, csy = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t b = __ballot(co[64 * k + lane] != 0);
        if ((tu4 >> k) & 1) {  // four 4x4 TUs of 16 coefficients (lane = 16 j + scan index)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t f = (uint32_t)((b >> (16 * j)) & 0xffffu);
                if (!f) continue;
                s.cbf_y16 |= (uint16_t)(1u << (4 * k + j));
                s.cbf_y4 |= (uint8_t)(1u << k);
                lsum += (uint32_t)(32 - __builtin_clz(f));
                csy |= 1u << (4 * k + j);
            }
        } else if (b) {
            s.cbf_y4 |= (uint8_t)(1u << k);
            lsum += (uint32_t)(64 - __builtin_clzll(b));
            uint32_t m = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) m |= ((b >> (16 * q)) & 0xffffu) ? 1u << q : 0u;
            csy |= m << (4 * k);
        }
    }
    s.cbf = s.cbf_y4 ? 1 : 0;
    s.last[0] = (uint8_t)(lsum ? (lsum > 256 ? 255 : lsum - 1) : 0);
    s.csbf_y = (uint16_t)csy;
#pragma unroll
    for (int comp = 0; comp < 2; ++comp) {
        const uint64_t b = __ballot(co[256 + 64 * comp + lane] != 0);
        uint32_t csum = 0, cm = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t f = (uint32_t)((b >> (16 * k)) & 0xffffu);
            if (f) {
                s.cbf_c4 |= (uint8_t)(1u << (4 * comp + k));
                csum += (uint32_t)(32 - __builtin_clz(f));
                cm |= 1u << k;
            }
        }
        if (cm) s.cbf |= (uint8_t)(2 << comp);
        s.last[1 + comp] = (uint8_t)(csum ? csum - 1 : 0);
        s.csbf_c[comp] = (uint8_t)cm;
    }
    return s;
}

struct SplitResult {
    int sse_full;
    int sse[3];
    uint32_t bits;
    int sse_y_full;   // luma only, whole CU (residual drop)
    uint32_t bits_y;  // tu_bits_est sum of the four luma TUs
    // per 8x8 luma node k: SSE over the node, SSE over its display area, tu_bits_est, levels coded
    int node_sse[4], node_disp[4], node_lv[4];
    uint32_t node_bits[4];
};
__device__ __forceinline__ SplitResult split_tus(TuBuf& t, const Mats& M, int qp, int qpc, bool valid, int16_t* lv,
                                                uint8_t* rec, int x0, int y0, int disp_w, int disp_h) {
    const int lane = threadIdx.x & 63;
    const int tk = lane >> 4, lbx = (tk & 1) * 8, lby = (tk >> 1) * 8, lbase = 64 * tk;  // luma TU of the lane
    const int ct = lane >> 3, comp = ct >> 2, ck = ct & 3;                                 // chroma TU of the lane
    const int cbx = (ck & 1) * 4, cby = (ck >> 1) * 4, cbase = 256 + 64 * comp + 16 * ck;
    // int16 stage views with the layouts of code_tus (aT[k][y], bT[x][k], a16[y][x] per TU)
    int16_t* aT = reinterpret_cast<int16_t*>(t.a);
    int16_t* a16 = reinterpret_cast<int16_t*>(t.a);
    int16_t* bT = reinterpret_cast<int16_t*>(t.b);
    // ---- forward stage 1 (rows)
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = (lane & 15) * 4 + j, y = idx >> 3, k = idx & 7;
            const int s = dot8(M.t8 + k * 8, t.res + (lby + y) * 16 + lbx);
            aT[lbase + k * 8 + y] = (int16_t)((s + 2) >> 2);
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = (lane & 7) * 2 + j, y = idx >> 2, k = idx & 3;
            const int s = dot4(M.t4 + k * 4, t.res + 256 + comp * 64 + (cby + y) * 8 + cbx);
            aT[cbase + k * 4 + y] = (int16_t)((s + 1) >> 1);
        }
    }
    wave_lds_sync();
    // ---- forward stage 2 (columns) + quantisation
    int ll[4] = {0, 0, 0, 0}, lc[2] = {0, 0};
    int sil[4], sic[2];
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = (lane & 15) * 4 + j, k2 = idx >> 3, k = idx & 7;
            const int s = dot8(M.t8 + k2 * 8, aT + lbase + k * 8);
            ll[j] = quant_coef((s + 256) >> 9, qp, 3, false);
            sil[j] = scan_index(3, k, k2);
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = (lane & 7) * 2 + j, k2 = idx >> 2, k = idx & 3;
            const int s = dot4(M.t4 + k2 * 4, aT + cbase + k * 4);
            lc[j] = quant_coef((s + 128) >> 8, qpc, 2, false);
            sic[j] = scan_index(2, k, k2);
        }
    } else {
        for (int j = 0; j < 4; ++j) sil[j] = 0;
        for (int j = 0; j < 2; ++j) sic[j] = 0;
    }
    // ---- decimation per TU
    {
        int nz = 0, mx = 0;
        for (int j = 0; j < 4; ++j) {
            nz += ll[j] != 0;
            mx = max(mx, abs(ll[j]));
        }
        if (tu_decimate(3, false, gsum<16>(nz), gmax<16>(mx)))
            for (int j = 0; j < 4; ++j) ll[j] = 0;
        nz = mx = 0;
        for (int j = 0; j < 2; ++j) {
            nz += lc[j] != 0;
            mx = max(mx, abs(lc[j]));
        }
        if (tu_decimate(2, false, gsum<8>(nz), gmax<8>(mx)))
            for (int j = 0; j < 2; ++j) lc[j] = 0;
    }
    // ---- trailing isolated +-1 trim per TU (tu_encode_t rule; a stopped TU stays stopped)
    {
        bool on_l = true, on_c = true;
        for (int it = 0; it < kTrimIters; ++it) {
            int last = -1;
            for (int j = 0; j < 4; ++j)
                if (ll[j]) last = max(last, sil[j]);
            last = gmax<16>(last);
            int prev = -1, lvv = 0;
            for (int j = 0; j < 4; ++j) {
                if (ll[j] && sil[j] < last) prev = max(prev, sil[j]);
                if (ll[j] && sil[j] == last) lvv = abs(ll[j]);
            }
            prev = gmax<16>(prev);
            lvv = gmax<16>(lvv);
            if (last < 0 || lvv != 1 || last - prev <= kTrimGap) on_l = false;
            if (on_l)
                for (int j = 0; j < 4; ++j)
                    if (sil[j] == last) ll[j] = 0;
            int lastc = -1;
            for (int j = 0; j < 2; ++j)
                if (lc[j]) lastc = max(lastc, sic[j]);
            lastc = gmax<8>(lastc);
            int prevc = -1, lvc = 0;
            for (int j = 0; j < 2; ++j) {
                if (lc[j] && sic[j] < lastc) prevc = max(prevc, sic[j]);
                if (lc[j] && sic[j] == lastc) lvc = abs(lc[j]);
            }
            prevc = gmax<8>(prevc);
            lvc = gmax<8>(lvc);
            if (lastc < 0 || lvc != 1 || lastc - prevc <= kTrimGap) on_c = false;
            if (on_c)
                for (int j = 0; j < 2; ++j)
                    if (sic[j] == lastc) lc[j] = 0;
        }
    }
    // ---- levels, dequantised values, per-TU counts and bit estimates
    int nzl = 0, nzc = 0, bl = 0, bc = 0;
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = (lane & 15) * 4 + j, k2 = idx >> 3, k = idx & 7;
            const int l = ll[j];
            lv[lbase + sil[j]] = (int16_t)l;
            bT[lbase + k * 8 + k2] = (int16_t)dequant_coef(l, qp, 3);
            if (l) {
                ++nzl;
                bl += 4 + 2 * (31 - __builtin_clz((uint32_t)abs(l)));
            }
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = (lane & 7) * 2 + j, k2 = idx >> 2, k = idx & 3;
            const int l = lc[j];
            lv[cbase + sic[j]] = (int16_t)l;
            bT[cbase + k * 4 + k2] = (int16_t)dequant_coef(l, qpc, 2);
            if (l) {
                ++nzc;
                bc += 4 + 2 * (31 - __builtin_clz((uint32_t)abs(l)));
            }
        }
    }
    nzl = gsum<16>(nzl);
    nzc = gsum<8>(nzc);
    bl = gsum<16>(bl);
    bc = gsum<8>(bc);
    SplitResult out;
    out.bits = (uint32_t)wsum(((lane & 15) == 0 ? (nzl ? bl + 4 : 1) : 0) + ((lane & 7) == 0 ? (nzc ? bc + 4 : 1) : 0));
    out.bits_y = (uint32_t)wsum((lane & 15) == 0 ? (nzl ? bl + 4 : 1) : 0);
    wave_lds_sync();
    // ---- inverse stage 1 (columns)
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = (lane & 15) * 4 + j, y = idx >> 3, x = idx & 7;
            const int s = dot8(M.tt8 + y * 8, bT + lbase + x * 8);
            a16[lbase + idx] = (int16_t)clip16((s + 64) >> 7);
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = (lane & 7) * 2 + j, y = idx >> 2, x = idx & 3;
            const int s = dot4(M.tt4 + y * 4, bT + cbase + x * 4);
            a16[cbase + idx] = (int16_t)clip16((s + 64) >> 7);
        }
    }
    wave_lds_sync();
    // ---- inverse stage 2 (rows) + reconstruction
    int sf = 0, sy = 0, sc = 0, syf = 0;
    if (valid) {
        for (int j = 0; j < 4; ++j) {
            const int idx = (lane & 15) * 4 + j, y = idx >> 3, x = idx & 7;
            const int s = dot8(M.tt8 + x * 8, a16 + lbase + y * 8);
            const int r = nzl ? (s + 2048) >> 12 : 0;
            const int o = (lby + y) * 16 + lbx + x, p = t.pred[o];
            const int v = clip255(p + r), e = p + t.res[o] - v;
            sf += e * e;
            syf += e * e;
            sy += (x0 + lbx + x < disp_w && y0 + lby + y < disp_h) ? e * e : 0;
            rec[o] = (uint8_t)v;
        }
        for (int j = 0; j < 2; ++j) {
            const int idx = (lane & 7) * 2 + j, y = idx >> 2, x = idx & 3;
            const int s = dot4(M.tt4 + x * 4, a16 + cbase + y * 4);
            const int r = nzc ? (s + 2048) >> 12 : 0;
            const int o = 256 + comp * 64 + (cby + y) * 8 + cbx + x, p = t.pred[o];
            const int v = clip255(p + r), e = p + t.res[o] - v;
            sf += e * e;
            sc += (2 * (x0 / 2 + cbx + x) < disp_w && 2 * (y0 / 2 + cby + y) < disp_h) ? e * e : 0;
            rec[o] = (uint8_t)v;
        }
    }
    out.sse_full = wsum(sf);
    out.sse_y_full = wsum(syf);
    out.sse[0] = wsum(sy);
    out.sse[1] = wsum(comp == 0 ? sc : 0);
    out.sse[2] = wsum(comp == 1 ? sc : 0);
    {  // per luma node: the 16-lane group sums, read from the group's first lane
        const int gs = gsum<16>(syf), gd = gsum<16>(sy);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            out.node_sse[k] = __builtin_amdgcn_readlane(gs, 16 * k);
            out.node_disp[k] = __builtin_amdgcn_readlane(gd, 16 * k);
            out.node_lv[k] = __builtin_amdgcn_readlane(nzl, 16 * k);
            out.node_bits[k] = (uint32_t)__builtin_amdgcn_readlane(nzl ? bl + 4 : 1, 16 * k);
        }
    }
    wave_lds_sync();
    return out;
}

// The 4x4 option of the split tree's luma nodes (split_encode's try4 on the CPU), whole wave: 4x4
// TU j16 = lane >> 2 (node k = j16 >> 2, TU j = j16 & 3 in z order), lane l4 = lane & 3 takes row l4
// of the forward row stage, column l4 of the column stage and row l4 of both inverse stages;
// decimation and the trailing trim per TU over its 4 lanes (tu_encode_t<2> rules).  Levels to lv4
// (node k TU j at 64k + 16j, scan order), reconstruction to rec4 (16x16 luma, TuBuf layout);
// per-node SSE (node / display area) and bits in the result.
struct Split4Result {
    int node_sse[4], node_disp[4];
    uint32_t node_bits[4];
};
__device__ __forceinline__ Split4Result split4_luma(TuBuf& t, const Mats& M, int qp, bool valid, int16_t* lv4,
                                                    uint8_t* rec4, int x0, int y0, int disp_w, int disp_h) {
    const int lane = threadIdx.x & 63, j16 = lane >> 2, l4 = lane & 3;
    const int k = j16 >> 2, j = j16 & 3;
    const int tx = (k & 1) * 8 + (j & 1) * 4, ty = (k >> 1) * 8 + (j >> 1) * 4;  // TU origin in the CU
    const int base = 16 * j16;
    int16_t* aT = reinterpret_cast<int16_t*>(t.a);
    int16_t* a16 = reinterpret_cast<int16_t*>(t.a);
    int16_t* bT = reinterpret_cast<int16_t*>(t.b);
    if (valid)  // forward stage 1 (rows): row l4, outputs kk
        for (int kk = 0; kk < 4; ++kk) {
            const int s = dot4(M.t4 + kk * 4, t.res + (ty + l4) * 16 + tx);
            aT[base + kk * 4 + l4] = (int16_t)((s + 1) >> 1);
        }
    wave_lds_sync();
    int ll[4] = {0, 0, 0, 0}, si[4] = {0, 0, 0, 0};
    if (valid)  // forward stage 2 (columns): column kk = l4, vertical frequency k2
        for (int k2 = 0; k2 < 4; ++k2) {
            const int s = dot4(M.t4 + k2 * 4, aT + base + l4 * 4);
            ll[k2] = quant_coef((s + 128) >> 8, qp, 2, false);
            si[k2] = scan_index(2, l4, k2);
        }
    {  // decimation per TU
        int nz = 0, mx = 0;
        for (int q = 0; q < 4; ++q) {
            nz += ll[q] != 0;
            mx = max(mx, abs(ll[q]));
        }
        if (tu_decimate(2, false, gsum<4>(nz), gmax<4>(mx)))
            for (int q = 0; q < 4; ++q) ll[q] = 0;
    }
    {  // trailing isolated +-1 trim per TU (a stopped TU stays stopped)
        bool on = true;
        for (int it = 0; it < kTrimIters; ++it) {
            int last = -1;
            for (int q = 0; q < 4; ++q)
                if (ll[q]) last = max(last, si[q]);
            last = gmax<4>(last);
            int prev = -1, lvv = 0;
            for (int q = 0; q < 4; ++q) {
                if (ll[q] && si[q] < last) prev = max(prev, si[q]);
                if (ll[q] && si[q] == last) lvv = abs(ll[q]);
            }
            prev = gmax<4>(prev);
            lvv = gmax<4>(lvv);
            if (last < 0 || lvv != 1 || last - prev <= kTrimGap) on = false;
            if (on)
                for (int q = 0; q < 4; ++q)
                    if (si[q] == last) ll[q] = 0;
        }
    }
    int nz = 0, bl = 0;
    if (valid)
        for (int k2 = 0; k2 < 4; ++k2) {
            const int l = ll[k2];
            lv4[64 * k + 16 * j + si[k2]] = (int16_t)l;
            bT[base + l4 * 4 + k2] = (int16_t)dequant_coef(l, qp, 2);
            if (l) {
                ++nz;
                bl += 4 + 2 * (31 - __builtin_clz((uint32_t)abs(l)));
            }
        }
    nz = gsum<4>(nz);
    bl = gsum<4>(bl);
    wave_lds_sync();
    if (valid)  // inverse stage 1 (columns): row y = l4 of the intermediate
        for (int x = 0; x < 4; ++x) {
            const int s = dot4(M.tt4 + l4 * 4, bT + base + x * 4);
            a16[base + l4 * 4 + x] = (int16_t)clip16((s + 64) >> 7);
        }
    wave_lds_sync();
    int sf = 0, sd = 0;
    if (valid)  // inverse stage 2 (rows) + reconstruction: row l4
        for (int x = 0; x < 4; ++x) {
            const int s = dot4(M.tt4 + x * 4, a16 + base + l4 * 4);
            const int r = nz ? (s + 2048) >> 12 : 0;
            const int o = (ty + l4) * 16 + tx + x, p = t.pred[o];
            const int v = clip255(p + r), e = p + t.res[o] - v;
            sf += e * e;
            sd += (x0 + tx + x < disp_w && y0 + ty + l4 < disp_h) ? e * e : 0;
            rec4[o] = (uint8_t)v;
        }
    Split4Result out;
    const int gs = gsum<16>(sf), gd = gsum<16>(sd);
    const int gb = gsum<16>(l4 == 0 ? (nz ? bl + 4 : 1) : 0);  // the node's four TUs
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        out.node_sse[q] = __builtin_amdgcn_readlane(gs, 16 * q);
        out.node_disp[q] = __builtin_amdgcn_readlane(gd, 16 * q);
        out.node_bits[q] = (uint32_t)__builtin_amdgcn_readlane(gb, 16 * q);
    }
    wave_lds_sync();
    return out;
}

__device__ __forceinline__ void fill_cu(CuInfo& c, const TuResult& r) {
    c.tu_split = 0;
    c.cbf_y4 = c.cbf_c4 = 0;
    c.est_bytes = 0;
    c.cbf = (uint8_t)((r.nz[0] ? 1 : 0) | (r.nz[1] ? 2 : 0) | (r.nz[2] ? 4 : 0));
    c.last[0] = (uint8_t)(r.last[0] < 0 ? 0 : r.last[0]);
    c.last[1] = (uint8_t)(r.last[1] < 0 ? 0 : r.last[1]);
    c.last[2] = (uint8_t)(r.last[2] < 0 ? 0 : r.last[2]);
    c.csbf_y = (uint16_t)r.csbf[0];
    c.csbf_c[0] = (uint8_t)r.csbf[1];
    c.csbf_c[1] = (uint8_t)r.csbf[2];
}

// ------------------------------------------------------------------ inter
__global__ __launch_bounds__(256) void k_hevc_inter(Geometry g, const HevcFrameState* __restrict__ fs,
                                                     const h264::MbInfo* __restrict__ mbs,
                                                     const uint8_t* __restrict__ src_y,
                                                     const uint8_t* __restrict__ src_uv, CuInfo* __restrict__ cus,
                                                     int16_t* __restrict__ coef, uint32_t* __restrict__ cost,
                                                     uint8_t* __restrict__ qp_coded) {
    __shared__ Mats M;
    __shared__ TuBuf tb[4];
    __shared__ unsigned long long part[3][4];
    __shared__ int16_t lv2[4][kCoefPerCu];  // split transform tree: levels and reconstruction
    __shared__ uint8_t rec2[4][384];
    __shared__ int16_t lv4[4][256];          // its 4x4 luma option (tu_split 2)
    __shared__ uint8_t rec4[4][256];
    __shared__ uint32_t unit_cost[4];
    fill_mats(M);
    __syncthreads();
    // one workgroup per 32x32 CTB, wave z = its unit in z order (the slice layout balances CTBs:
    // the workgroup adds up the CTB's cost)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bid = blockIdx.x;
    const int cw = ctb_cols(g.mb_w);
    const int ux = 2 * (bid % cw) + (wave & 1), uy = 2 * (bid / cw) + (wave >> 1);
    const bool valid = ux < g.mb_w && uy < g.mb_h;
    const int i = valid ? uy * g.mb_w + ux : 0;
    const int x = valid ? ux : 0, y = valid ? uy : 0;
    const int x0 = x * 16, y0 = y * 16;
    TuBuf& t = tb[wave];
    int mvx = 0, mvy = 0, lsad = 0;
    int tsad = 0;           // this lane's share of sum |src - previous src| (temporal class, aq 3)
    int dpf = 0, dpm = 0;   // sum res^2 of the lane's luma samples: whole CU / display area
    uint32_t pred_px = 0;   // the lane's 4 luma prediction samples (residual drop)
    int dcp[2] = {0, 0};    // sum (src - pred)^2 of the lane's chroma samples in the display area
    if (valid) {
        // the CU's vector is wave-uniform: scalar registers, so the filter taps are scalar too
        mvx = __builtin_amdgcn_readfirstlane(mbs[i].mvx);
        mvy = __builtin_amdgcn_readfirstlane(mbs[i].mvy);
        // luma: 4 samples per lane from the edge-padded reference (|mv| stays inside the pad),
        // separable: each of the (up to 8) reference rows is loaded once (11 bytes) and filtered
        // horizontally for all 4 samples before the vertical taps
        const int r = lane >> 2, cb = (lane & 3) * 4;
        const uint8_t* F = fs->hp_f;
        const int P = fs->hp_pitch;
        const int fx = mvx & 3, fy = mvy & 3;
        const int xi = x0 + cb + (mvx >> 2), yi = y0 + r + (mvy >> 2);
        int vv[4];
        if (!fx && !fy) {
            const uint8_t* row = F + yi * P + xi;
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[j] = row[j] << 6;
        } else if (!fy) {
            const uint8_t* row = F + yi * P + xi - 3;
            int px[11];
#pragma unroll
            for (int q = 0; q < 11; ++q) px[q] = row[q];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int v = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) v += kLumaTap[fx][k] * px[j + k];
                vv[j] = v;
            }
        } else if (!fx) {
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[j] = 0;
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const uint8_t* row = F + (yi + n - 3) * P + xi;
#pragma unroll
                for (int j = 0; j < 4; ++j) vv[j] += kLumaTap[fy][n] * row[j];
            }
        } else {
            int sv[4] = {0, 0, 0, 0};
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const uint8_t* row = F + (yi + n - 3) * P + xi - 3;
                int px[11];
#pragma unroll
                for (int q = 0; q < 11; ++q) px[q] = row[q];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int h = 0;
#pragma unroll
                    for (int k = 0; k < 8; ++k) h += kLumaTap[fx][k] * px[j + k];
                    sv[j] += kLumaTap[fy][n] * h;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[j] = sv[j] >> 6;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = clip255((vv[j] + 32) >> 6);
            const int d = (int)src_y[(size_t)(y0 + r) * g.pitch + x0 + cb + j] - p;
            t.pred[r * 16 + cb + j] = (uint8_t)p;
            t.res[r * 16 + cb + j] = (int16_t)d;
            lsad += d < 0 ? -d : d;
            pred_px |= (uint32_t)p << (8 * j);
            dpf += d * d;
            dpm += (x0 + cb + j < g.width && y0 + r < g.height) ? d * d : 0;
        }
        if (fs->aq >= 3) {
            // temporal class: the source against the previous source displaced by the vector's
            // integer part; this CU's source becomes the next frame's previous source
            const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y0 + r) * g.pitch + x0 + cb);
            for (int j = 0; j < 4; ++j)
                tsad += abs((int)((sw >> (8 * j)) & 0xff) - h264::ref_px(fs->prev_src, g.pitch, g.coded_w, g.coded_h,
                                                                          x0 + cb + j + (mvx >> 2), y0 + r + (mvy >> 2)));
            *reinterpret_cast<uint32_t*>(fs->save_src + (size_t)(y0 + r) * g.pitch + x0 + cb) = sw;
        }
        // chroma: one sample per lane and component
        const int rc = lane >> 3, cc = lane & 7;
        const int xc = x0 / 2 + cc, yc = y0 / 2 + rc;
        for (int comp = 0; comp < 2; ++comp) {
            const int p = chroma_mc(fs->ref_uv, g.pitch, g.coded_w / 2, g.coded_h / 2, comp, xc, yc, mvx, mvy);
            const int s = src_uv[(size_t)yc * g.pitch + 2 * xc + comp];
            t.pred[256 + comp * 64 + rc * 8 + cc] = (uint8_t)p;
            t.res[256 + comp * 64 + rc * 8 + cc] = (int16_t)(s - p);
            dcp[comp] = (2 * xc < g.width && 2 * yc < g.height) ? (s - p) * (s - p) : 0;
        }
    }
    const int tcls = h264::temporal_class((uint32_t)wsum(tsad), mvx == 0 && mvy == 0);  // vector wave-uniform
    const int qp = h264::mb_qp_for(fs->qp, (uint32_t)wsum(lsad), tcls, fs->aq);  // wave-uniform
    const int qpc = chroma_qp(qp, fs->chroma_qp_offset);
    // changing content (aq 3): chroma residual dropped, luma kept only if it pays for its bits
    const bool changing = fs->aq >= 3 && tcls == h264::kTcChanging;
    const bool cdrop = changing && !fs->chroma_keep;  // wave-uniform
    if (cdrop && valid) {
        const int rc = lane >> 3, cc = lane & 7;
        for (int comp = 0; comp < 2; ++comp) t.res[256 + comp * 64 + rc * 8 + cc] = 0;
    }
    wave_lds_sync();  // from here on every wave works alone (wave-local syncs, per-wave LDS)
    int16_t* co = coef + (size_t)(valid ? i : 0) * kCoefPerCu;
    // option 1, one 16x16 luma TU (writes its levels and reconstruction; t.pred keeps the prediction)
    const TuResult r = code_tus<true>(t, M, qp, qpc, false, valid, co, fs->rec_y, g.pitch, fs->rec_uv, x0, y0,
                                      g.width, g.height);
    // option 2, the split transform tree (split_encode of the CPU encoder), whole wave -- only
    // when option 1 coded something (split_worth_trying, as the CPU encoder)
    const bool try_split = fs->tu_split != 0 && valid && split_worth_trying(r.nz[0] + r.nz[1] + r.nz[2]);  // wave-uniform
    SplitResult r2 = {};
    if (try_split)
        r2 = split_tus(t, M, qp, qpc, valid, lv2[wave], rec2[wave], x0, y0, g.width, g.height);
    // tu_split 2: every node whose 8x8 TU coded a level may become four 4x4 TUs (split_encode try4)
    int tu4 = 0;
    if (try_split && fs->tu_split >= 2 &&
        split_worth_trying(r2.node_lv[0] + r2.node_lv[1] + r2.node_lv[2] + r2.node_lv[3])) {  // wave-uniform
        const Split4Result r4 = split4_luma(t, M, qp, valid, lv4[wave], rec4[wave], x0, y0, g.width, g.height);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!split_worth_trying(r2.node_lv[k])) continue;
            if (!choose_split((uint64_t)r2.node_sse[k], r2.node_bits[k], (uint64_t)r4.node_sse[k], r4.node_bits[k], qp))
                continue;
            tu4 |= 1 << k;
            r2.sse_full += r4.node_sse[k] - r2.node_sse[k];
            r2.sse_y_full += r4.node_sse[k] - r2.node_sse[k];
            r2.sse[0] += r4.node_disp[k] - r2.node_disp[k];
            r2.bits += r4.node_bits[k] - r2.node_bits[k];
            r2.bits_y += r4.node_bits[k] - r2.node_bits[k];
            // node k's levels and luma reconstruction from the 4x4 option
            lv2[wave][64 * k + lane] = lv4[wave][64 * k + lane];
            {
                const int ry = (k >> 1) * 8 + (lane >> 3), rx = (k & 1) * 8 + (lane & 7);
                rec2[wave][ry * 16 + rx] = rec4[wave][ry * 16 + rx];
            }
        }
        wave_lds_sync();
    }
    const int sse2 = r2.sse_full, bits2 = (int)r2.bits;
    const int sse2y = r2.sse[0], sse2u = r2.sse[1], sse2v = r2.sse[2];
    const bool split = try_split &&
                       choose_split((uint64_t)r.sse_full, r.bits, (uint64_t)sse2, (uint32_t)bits2, qp);  // wave-uniform
    if (split) {  // the split tree wins: overwrite option 1's levels and reconstruction
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int k = lane; k < kCoefPerCu; k += 64) co[k] = lv2[wave][k];
        const int yy = lane >> 2, xb = (lane & 3) * 4;
        uint32_t packed = 0;
        for (int j = 0; j < 4; ++j) packed |= (uint32_t)rec2[wave][yy * 16 + xb + j] << (8 * j);
        *reinterpret_cast<uint32_t*>(fs->rec_y + (size_t)(y0 + yy) * g.pitch + x0 + xb) = packed;
        const int rc = lane >> 3, cc = lane & 7;
        for (int comp = 0; comp < 2; ++comp)
            fs->rec_uv[(size_t)(y0 / 2 + rc) * g.pitch + 2 * (x0 / 2 + cc) + comp] = rec2[wave][256 + comp * 64 + rc * 8 + cc];
    }
    // rate-distortion residual drop of changing content (h264_mb.h drop_luma_for): the luma
    // residual must lower the distortion by more than lambda * (estimated bits)
    const long long d_pred = wsum(dpf);
    const bool drop = cdrop && valid &&
                      d_pred - (long long)(split ? r2.sse_y_full : r.sse_y_full) <
                          (long long)h264::lambda_sse(qp) * (long long)(split ? r2.bits_y : r.bits_y);  // wave-uniform
    const int dp_disp = wsum(dpm);
    const int dcp_u = wsum(dcp[0]), dcp_v = wsum(dcp[1]);  // chroma distortion when its residual is dropped
    if (drop) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // after this lane's coded levels / reconstruction
        for (int k = lane; k < 256; k += 64) co[k] = 0;
        *reinterpret_cast<uint32_t*>(fs->rec_y + (size_t)(y0 + (lane >> 2)) * g.pitch + x0 + (lane & 3) * 4) = pred_px;
    }
    if (lane == 0) {
        part[0][wave] = valid ? (unsigned long long)(drop ? dp_disp : (split ? sse2y : r.sse[0])) : 0ull;
        part[1][wave] = valid ? (unsigned long long)(cdrop ? dcp_u : (split ? sse2u : r.sse[1])) : 0ull;
        part[2][wave] = valid ? (unsigned long long)(cdrop ? dcp_v : (split ? sse2v : r.sse[2])) : 0ull;
    }
    SplitSummary ss = {};
    if (split) ss = split_summary_wave(lv2[wave], lane, tu4);  // wave-uniform branch
    if (valid && lane == 0) {
        CuInfo c{};
        c.type = kCuAmvp;
        c.intra_mode = 1;
        c.qp = (uint8_t)qp;
        c.mvx = (int16_t)mvx;
        c.mvy = (int16_t)mvy;
        c.mvdx = c.mvdy = 0;
        c.mvp_idx = 0;
        fill_cu(c, r);
        if (fs->tu_split) {
            c.tu_split = split ? 2 : 1;
            if (split) ss.apply(c);
        }
        if (drop) {  // no residual left (chroma was dropped before coding): cu_summarise of zeros
            c.tu_split = fs->tu_split ? 1 : 0;
            c.cbf = c.cbf_y4 = c.cbf_c4 = 0;
            c.tu4 = 0;
            c.cbf_y16 = 0;
            c.last[0] = c.last[1] = c.last[2] = 0;
            c.csbf_y = 0;
            c.csbf_c[0] = c.csbf_c[1] = 0;
        }
        set_est_bytes(c, split ? r2.bits : r.bits);
        c.ct = 1;
        cus[i] = c;  // skip / merge / AMVP and the coding tree are decided by k_hevc_decide once the slices are laid out
        qp_coded[i] = c.cbf ? c.qp : (uint8_t)255;
        unit_cost[wave] = cu_cost(c);
    }
    if (!valid && lane == 0) unit_cost[wave] = 0u;
    __syncthreads();
    if (threadIdx.x == 0) cost[bid] = unit_cost[0] + unit_cost[1] + unit_cost[2] + unit_cost[3];
    if (threadIdx.x < 3) {
        const int c = threadIdx.x;
        fs->sse_part[c * h264::kSsePartStride + bid] = part[c][0] + part[c][1] + part[c][2] + part[c][3];
    }
}

// ------------------------------------------------------------------ intra
// Per-wave reference state of the CU being predicted.
struct IntraRefs {
    uint8_t lpx[16], tpx[16], trx[16];
    uint8_t lc[2][8], tc[2][8], trc[2][8];
    int corner, corner_c[2];
    int L[33], T[33], LF[33], TF[33];  // luma refs (unfiltered / planar-filtered)
    int Lc[2][17], Tc[2][17];
    int dc, dcc[2];
};

// Sample (x, y) of the prediction of any intra mode; equals intra_predict().  L / T: the
// references (index 0 = corner), LF / TF the [1 2 1]-filtered ones (8.4.4.2.3, luma only).
__device__ __forceinline__ int pred_sample(int mode, int log2n, bool luma, const int* L, const int* T, const int* LF,
                                           const int* TF, int dc, int x, int y) {
    const int N = 1 << log2n;
    if (mode >= 2 && mode != 10 && mode != 26) {  // angular (8.4.4.2.6)
        const int d1 = mode > 26 ? mode - 26 : 26 - mode, d2 = mode > 10 ? mode - 10 : 10 - mode;
        const int thres = N == 8 ? 7 : (N == 16 ? 1 : 0);
        const bool filt = luma && N != 4 && (d1 < d2 ? d1 : d2) > thres;
        const bool vert = mode >= 18;
        const int* mainr = vert ? (filt ? TF : T) : (filt ? LF : L);
        const int* side = vert ? (filt ? LF : L) : (filt ? TF : T);
        const int angle = kIntraAngle[mode];
        const int a = vert ? y : x, b = vert ? x : y;  // a: distance along the prediction, b: across it
        const int pos = (a + 1) * angle, idx = pos >> 5, fact = pos & 31;
        const int k = b + idx + 1;
        // ref[k] for k >= 0 is the main array; negative k (negative angles) projects onto the side
        // array through the inverse angle, as intra_predict() extends ref[]
        const int ia = angle < 0 ? inv_angle(angle) : 0;
        const int r0 = k >= 0 ? mainr[k] : side[(k * ia + 128) >> 8];
        if (!fact) return r0;
        const int r1 = k + 1 >= 0 ? mainr[k + 1] : side[((k + 1) * ia + 128) >> 8];
        return ((32 - fact) * r0 + fact * r1 + 16) >> 5;
    }
    if (mode == 0)
        return ((N - 1 - x) * LF[1 + y] + (x + 1) * TF[1 + N] + (N - 1 - y) * TF[1 + x] + (y + 1) * LF[1 + N] + N) >>
               (log2n + 1);
    if (mode == 1) {
        if (luma && N < 32) {
            if (x == 0 && y == 0) return (L[1] + 2 * dc + T[1] + 2) >> 2;
            if (y == 0) return (T[1 + x] + 3 * dc + 2) >> 2;
            if (x == 0) return (L[1 + y] + 3 * dc + 2) >> 2;
        }
        return dc;
    }
    if (mode == 26) return (luma && x == 0) ? clip255(T[1] + ((L[1 + y] - L[0]) >> 1)) : T[1 + x];
    return (luma && y == 0) ? clip255(L[1] + ((T[1 + x] - T[0]) >> 1)) : L[1 + y];  // mode 10
}

// Reference sample i (0 .. 4N, the spec's search order from p[-1][2N-1] up to the corner and
// right to p[2N-1][-1]) after 8.4.4.2.2 substitution, in closed form over the five segments
// (bottom-left, left, corner, top, top-right; bit s of avl = segment s available): an
// unavailable segment takes the last sample of the nearest available segment before it, or,
// when none precedes, the first sample of the first available one; none available: 128.
__device__ __forceinline__ int ref_subst(int i, int N, int avl, const uint8_t* lpx, const uint8_t* tpx,
                                         const uint8_t* trx, int corner) {
    if (avl == 0) return 128;
    const int n2 = 2 * N;
    const int seg = i < N ? 0 : (i < n2 ? 1 : (i == n2 ? 2 : (i <= 3 * N ? 3 : 4)));
    int j = i;
    if (!((avl >> seg) & 1)) {
        const int below = avl & ((1 << seg) - 1);
        if (below) {
            const int p = 31 - __clz(below);  // last sample of segment p
            j = p == 0 ? N - 1 : (p == 1 ? n2 - 1 : (p == 2 ? n2 : (p == 3 ? 3 * N : 4 * N)));
        } else {
            const int f = __ffs(avl) - 1;  // first sample of segment f
            j = f == 0 ? 0 : (f == 1 ? N : (f == 2 ? n2 : (f == 3 ? n2 + 1 : 3 * N + 1)));
        }
    }
    // j lies in an available segment (never the bottom-left here)
    if (j < n2) return lpx[n2 - 1 - j];
    if (j == n2) return corner;
    if (j <= 3 * N) return tpx[j - n2 - 1];
    return trx[j - 3 * N - 1];
}

// ref_subst's source index: the search-order position whose sample reference i takes (-1: none
// available, the value 128)
__device__ __forceinline__ int ref_subst_idx(int i, int N, int avl) {
    if (avl == 0) return -1;
    const int n2 = 2 * N;
    const int seg = i < N ? 0 : (i < n2 ? 1 : (i == n2 ? 2 : (i <= 3 * N ? 3 : 4)));
    if ((avl >> seg) & 1) return i;
    const int below = avl & ((1 << seg) - 1);
    if (below) {
        const int p = 31 - __clz(below);
        return p == 0 ? N - 1 : (p == 1 ? n2 - 1 : (p == 2 ? n2 : (p == 3 ? 3 * N : 4 * N)));
    }
    const int f = __ffs(avl) - 1;
    return f == 0 ? 0 : (f == 1 ? N : (f == 2 ? n2 : (f == 3 ? n2 + 1 : 3 * N + 1)));
}

// References of the four 8x8 TUs of a split intra unit (hevc_core.h split_tu_avl): raw samples (left
// then below-left, top, top-right, corner), substituted L / T, the [1 2 1]-filtered LF / TF, DC.
struct SplitRefs {
    uint8_t lp[4][16], tp[4][8], tr[4][8];
    int corner[4];
    int L[4][17], T[4][17], LF[4][17], TF[4][17];
    int dc[4];
};
// Substitution, filtering and DC of SplitRefs whose raw samples are in place (whole wave; ends
// with the wave's LDS hand-off).
__device__ __forceinline__ void split_refs_finish(SplitRefs& S, bool al, bool ac, bool at, bool atr, int lane) {
    for (int i = lane; i < 4 * 33; i += 64) {
        const int k = i / 33, q = i - k * 33;
        const int v = ref_subst(q, 8, split_tu_avl(k, al, ac, at, atr), S.lp[k], S.tp[k], S.tr[k], S.corner[k]);
        if (q < 16) S.L[k][16 - q] = v;
        else if (q == 16) S.L[k][0] = S.T[k][0] = v;
        else S.T[k][q - 16] = v;
    }
    wave_lds_sync();
    for (int i = lane; i < 4 * 17; i += 64) {
        const int k = i / 17, q = i - k * 17;
        if (q == 0) {
            S.LF[k][0] = S.TF[k][0] = (S.L[k][1] + 2 * S.L[k][0] + S.T[k][1] + 2) >> 2;
        } else if (q == 16) {
            S.LF[k][16] = S.L[k][16];
            S.TF[k][16] = S.T[k][16];
        } else {
            S.LF[k][q] = (S.L[k][q + 1] + 2 * S.L[k][q] + S.L[k][q - 1] + 2) >> 2;
            S.TF[k][q] = (S.T[k][q + 1] + 2 * S.T[k][q] + S.T[k][q - 1] + 2) >> 2;
        }
    }
    {
        const int k = lane >> 4, q = lane & 15;
        const int sum = gsum<16>(q < 8 ? S.L[k][1 + q] : S.T[k][1 + q - 8]);
        if (q == 0) S.dc[k] = (sum + 8) >> 4;
    }
    wave_lds_sync();
}

// ------------------------------------------------------------------ intra mode decision (I)
// Open-loop, every unit of an I picture at once (one wave per unit, a workgroup per CTB): the
// modes predicted from the *source* neighbours with the decoder's z-order availability (never the
// below-left; a CTB's first unit keeps to bl_safe_modes, as k_hevc_intra reconstructs it before
// its below-left), scored by 4x4 Hadamard SATD + lambda * mode bits, searched coarse-to-fine
// (intra_mode_search: at most 15 of the 35 modes) -- hevc_cpu.cpp
// intra_decide_mode.  With intra splits on, the modes are searched again for four 8x8 TUs predicted
// from the source (split_tu_avl), and kIntraSplitFlag is set with that mode when intra_split_wins.  The IDR wavefront
// (k_hevc_intra) then only reconstructs.
__global__ __launch_bounds__(256) void k_hevc_intra_modes(Geometry g, const HevcFrameState* __restrict__ fs,
                                                           const uint8_t* __restrict__ src_y,
                                                           uint8_t* __restrict__ imode) {
    __shared__ IntraRefs rf[4];
    __shared__ SplitRefs srf[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bid = blockIdx.x, cw = ctb_cols(g.mb_w);
    const int x = 2 * (bid % cw) + (wave & 1), y = 2 * (bid / cw) + (wave >> 1);
    if (x >= g.mb_w || y >= g.mb_h) return;  // wave-uniform; no workgroup barrier below
    IntraRefs& R = rf[wave];
    const int sr = fs->slice_rows, z = ((y & 1) << 1) | (x & 1);
    int xb, xe;
    i_seg_range(x, fs->i_seg_w, g.mb_w, xb, xe);
    const bool al = x > xb, at = (y % sr) != 0, atr = at && x + 1 < xe && z != 3, ac = at && x > xb;
    const bool bl_pending = z == 0 && x > xb && y + 1 < g.mb_h;
    const int x0 = x * 16, y0 = y * 16, P = g.pitch;
    if (lane < 16) {
        R.lpx[lane] = al ? src_y[(size_t)(y0 + lane) * P + x0 - 1] : 0;
        R.tpx[lane] = at ? src_y[(size_t)(y0 - 1) * P + x0 + lane] : 0;
        R.trx[lane] = atr ? src_y[(size_t)(y0 - 1) * P + x0 + 16 + lane] : 0;
    } else if (lane == 16) {
        R.corner = ac ? src_y[(size_t)(y0 - 1) * P + x0 - 1] : 0;
    }
    wave_lds_sync();
    const int avl = (al ? 2 : 0) | (ac ? 4 : 0) | (at ? 8 : 0) | (atr ? 16 : 0);
    for (int i = lane; i <= 64; i += 64) {
        const int v = ref_subst(i, 16, avl, R.lpx, R.tpx, R.trx, R.corner);
        if (i < 32) R.L[32 - i] = v;
        else if (i == 32) R.L[0] = R.T[0] = v;
        else R.T[i - 32] = v;
    }
    wave_lds_sync();
    if (lane <= 32) {
        const int k = lane;
        if (k == 0) {
            R.LF[0] = R.TF[0] = (R.L[1] + 2 * R.L[0] + R.T[1] + 2) >> 2;
        } else if (k == 32) {
            R.LF[32] = R.L[32];
            R.TF[32] = R.T[32];
        } else {
            R.LF[k] = (R.L[k + 1] + 2 * R.L[k] + R.L[k - 1] + 2) >> 2;
            R.TF[k] = (R.T[k + 1] + 2 * R.T[k] + R.T[k - 1] + 2) >> 2;
        }
    }
    const int sdc = wsum(lane < 16 ? R.L[1 + lane] + R.T[1 + lane] : 0);
    if (lane == 0) R.dc = (sdc + 16) >> 5;
    wave_lds_sync();
    // 4x4 Hadamard SATD of all sixteen 4x4 blocks of the unit on the matrix cores: with the
    // residual R (16 x 16) and H16 = diag(H4, H4, H4, H4) (H4 the order-4 Hadamard matrix,
    // symmetric), S = H16 R H16 holds every block's transform, SATD = sum |S|.  Two
    // v_mfma_f32_16x16x16_f16 per mode: T = R H16 (A = R), then S = H16 T, whose B operand layout
    // (lane l: rows 4(l>>4)..+3 of column l&15) is exactly T's accumulator layout, so T goes
    // across as four f16 conversions.  Exact: |R| <= 255 and |T| <= 1020 are integers f16 holds,
    // S (<= 4080) accumulates in f32.  The lane computes the residual of row l & 15, columns
    // 4 (l >> 4) .. + 3 -- the A operand's layout.
    typedef _Float16 mf_h4 __attribute__((ext_vector_type(4)));
    typedef float mf_f4 __attribute__((ext_vector_type(4)));
    const int r = lane & 15, cb = (lane >> 4) * 4;
    const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y0 + r) * P + x0 + cb);
    mf_h4 hm;  // H16[l & 15][4 (l >> 4) + j]: the B operand of the first product, the A of the second
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = lane & 15, k = cb + j;
        // H4[a][b] = (-1)^(popcount(a & b)) for the order a = {++++, +-+-, ++--, +--+}
        const int sgn = __popc((row & 3) & (k & 3)) & 1 ? -1 : 1;
        hm[j] = (_Float16)((row >> 2) == (k >> 2) ? sgn : 0);
    }
    const mf_f4 zero = {0.f, 0.f, 0.f, 0.f};
    const int lambda = h264::lambda_sad(fs->qp);
    const uint64_t safe = fs->bl_safe;
    auto cost = [&](int m) {
        if (bl_pending && !((safe >> m) & 1)) return kIntraNoMode;  // wave-uniform
        mf_h4 a;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            a[j] = (_Float16)((int)((sw >> (8 * j)) & 0xff) -
                              pred_sample(m, 4, true, R.L, R.T, R.LF, R.TF, R.dc, cb + j, r));
        const mf_f4 t = __builtin_amdgcn_mfma_f32_16x16x16f16(a, hm, zero, 0, 0, 0);
        mf_h4 tb;
#pragma unroll
        for (int i = 0; i < 4; ++i) tb[i] = (_Float16)t[i];
        const mf_f4 sm = __builtin_amdgcn_mfma_f32_16x16x16f16(hm, tb, zero, 0, 0, 0);
        const int sad = (int)(__builtin_fabsf(sm[0]) + __builtin_fabsf(sm[1]) + __builtin_fabsf(sm[2]) +
                              __builtin_fabsf(sm[3]));
        return wsum(sad) + lambda * intra_mode_bits(m, 1, 1);
    };
    const int best = intra_mode_search(cost);  // coarse-to-fine: at most 15 of the 35 modes
    int out = best;
    const int cost16 = cost(best);
    if (fs->depth_intra > 0 && intra_split_possible(cost16, lambda)) {  // the split tree's own mode search (wave-uniform)
        SplitRefs& S = srf[wave];
        for (int i = lane; i < 4 * 33; i += 64) {  // raw references of the four TUs, from the source
            const int k = i / 33, q = i - k * 33;
            const int bx = x0 + (k & 1) * 8, by = y0 + (k >> 1) * 8;
            const int avl = split_tu_avl(k, al, ac, at, atr);
            if (q < 16) {  // left (q < 8), below-left
                S.lp[k][q] = (avl & (q < 8 ? 2 : 1)) ? src_y[(size_t)(by + q) * P + bx - 1] : 0;
            } else if (q < 24) {
                S.tp[k][q - 16] = (avl & 8) ? src_y[(size_t)(by - 1) * P + bx + q - 16] : 0;
            } else if (q < 32) {
                S.tr[k][q - 24] = (avl & 16) ? src_y[(size_t)(by - 1) * P + bx + 8 + q - 24] : 0;
            } else {
                S.corner[k] = (avl & 4) ? src_y[(size_t)(by - 1) * P + bx - 1] : 0;
            }
        }
        wave_lds_sync();
        split_refs_finish(S, al, ac, at, atr, lane);
        const int kq = ((r >> 3) << 1) | (cb >> 3);  // the lane's four samples lie in one TU
        const uint64_t safe_s = fs->bl_safe_split;
        auto cost_split = [&](int m) {
            if (bl_pending && !((safe_s >> m) & 1)) return kIntraNoMode;  // wave-uniform
            mf_h4 a;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                a[j] = (_Float16)((int)((sw >> (8 * j)) & 0xff) - pred_sample(m, 3, true, S.L[kq], S.T[kq], S.LF[kq],
                                                                               S.TF[kq], S.dc[kq], (cb + j) & 7, r & 7));
            const mf_f4 t = __builtin_amdgcn_mfma_f32_16x16x16f16(a, hm, zero, 0, 0, 0);
            mf_h4 tb;
#pragma unroll
            for (int i = 0; i < 4; ++i) tb[i] = (_Float16)t[i];
            const mf_f4 sm = __builtin_amdgcn_mfma_f32_16x16x16f16(hm, tb, zero, 0, 0, 0);
            const int sad = (int)(__builtin_fabsf(sm[0]) + __builtin_fabsf(sm[1]) + __builtin_fabsf(sm[2]) +
                                  __builtin_fabsf(sm[3]));
            return wsum(sad) + lambda * intra_mode_bits(m, 1, 1);
        };
        const int best_s = intra_mode_search(cost_split);
        if (intra_split_wins(cost16, cost_split(best_s), lambda)) out = best_s | kIntraSplitFlag;
    }
    if (lane == 0) imode[y * g.mb_w + x] = (uint8_t)out;
}

// A split intra unit (kIntraSplitFlag) in the IDR wavefront, by its wave alone (wave-local LDS
// hand-offs): TU k = 0..3 in z order, each its 8x8 luma (lane = sample y * 8 + x) and its two 4x4
// chroma TUs (lanes 0..31: component lane >> 4, sample (lane >> 2) & 3, lane & 3) -- references from
// the unit's neighbours (R) and the reconstruction of the TUs before it (t.pred), prediction in the
// unit's mode, then forward transform, quantisation (intra: no decimation, no trim), levels in the
// mode's scan order, inverse transform and reconstruction into t.pred / rec -- as tu_encode_t<3> /
// <2> of the CPU encoder's analyse_intra.  src: the unit's source (t.pred layout); lv: LDS copy of
// the unit's levels (CU layout); the raw references go through S.
struct SplitIntraResult {
    int sse[3];
    uint32_t bits;  // cu_bits_est of the split tree
};
__device__ SplitIntraResult split_intra_code(TuBuf& t, SplitRefs& S, const IntraRefs& R, const Mats& M,
                                             const uint8_t* src, int16_t* lv, int mode, int qp, int qpc, bool al,
                                             bool ac, bool at, bool atr, int16_t* coef, uint8_t* rec_y,
                                             uint8_t* rec_uv, int pitch, int x0, int y0, int disp_w, int disp_h) {
    const int lane = threadIdx.x & 63;
    const int scan = intra_scan_idx(mode);
    const int ly = lane >> 3, lx = lane & 7;                            // luma sample / coefficient
    const int comp = (lane >> 4) & 1, cy = (lane >> 2) & 3, cx = lane & 3;  // chroma (lanes < 32)
    const bool cl = lane < 32;
    int16_t* aT = reinterpret_cast<int16_t*>(t.a);  // stage buffers: luma [0, 64), chroma 64 + 16 comp
    int16_t* bT = reinterpret_cast<int16_t*>(t.b);
    int sse_y = 0, sse_c = 0;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
        const int bx = (k & 1) * 8, by = (k >> 1) * 8, cbx = bx >> 1, cby = by >> 1;
        const int avl = split_tu_avl(k, al, ac, at, atr);
        // ---- references in one pass: lane i < 33 takes luma reference i (ref_subst's search order:
        // below-left bottom-up, left, corner, top, top-right), i >= 33 chroma; each lane fetches its
        // substituted sample straight from the neighbours / the unit's reconstruction, the luma [1 2 1]
        // filter takes the neighbours in search order by lane shuffles (the ends stay unfiltered; at
        // the corner the filter is the same three-tap form), the DC sums are wave sums
        int dcl = 0, dcc0 = 0, dcc1 = 0;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            const int i = lane + 64 * pass;
            int v = 0;
            if (i < 33) {
                const int j = ref_subst_idx(i, 8, avl);
                if (j < 0) {
                    v = 128;
                } else if (j < 16) {  // left (q < 8) / below-left (TU 0 only) sample q
                    const int q = 15 - j;
                    v = q < 8 ? (bx == 0 ? R.lpx[by + q] : t.pred[(by + q) * 16 + bx - 1]) : R.lpx[q];
                } else if (j == 16) {
                    v = k == 0 ? R.corner : (k == 1 ? R.tpx[7] : (k == 2 ? R.lpx[7] : t.pred[7 * 16 + 7]));
                } else if (j <= 24) {
                    const int c = j - 17;
                    v = by == 0 ? R.tpx[bx + c] : t.pred[7 * 16 + bx + c];
                } else {
                    const int c = j - 25;
                    v = k == 0 ? R.tpx[8 + c] : (k == 1 ? R.trx[c] : t.pred[7 * 16 + 8 + c]);
                }
            } else if (i < 33 + 34) {
                const int c = (i - 33) / 17, q = (i - 33) - c * 17;
                const int j = ref_subst_idx(q, 4, avl);
                const uint8_t* up = t.pred + 256 + c * 64;
                if (j < 0) {
                    v = 128;
                } else if (j < 8) {
                    const int r = 7 - j;
                    v = r < 4 ? (cbx == 0 ? R.lc[c][cby + r] : up[(cby + r) * 8 + cbx - 1]) : R.lc[c][r];
                } else if (j == 8) {
                    v = k == 0 ? R.corner_c[c] : (k == 1 ? R.tc[c][3] : (k == 2 ? R.lc[c][3] : up[3 * 8 + 3]));
                } else if (j <= 12) {
                    const int d = j - 9;
                    v = cby == 0 ? R.tc[c][cbx + d] : up[3 * 8 + cbx + d];
                } else {
                    const int d = j - 13;
                    v = k == 0 ? R.tc[c][4 + d] : (k == 1 ? R.trc[c][d] : up[3 * 8 + 4 + d]);
                }
                if (q < 8) S.L[1 + c][8 - q] = v;
                else if (q == 8) S.L[1 + c][0] = S.T[1 + c][0] = v;
                else S.T[1 + c][q - 8] = v;
            }
            if (pass == 0) {
                const int vm = __shfl_up(v, 1, 64), vp = __shfl_down(v, 1, 64);
                if (i < 33) {
                    const int f = (i == 0 || i == 32) ? v : (vm + 2 * v + vp + 2) >> 2;
                    if (i < 16) {
                        S.L[0][16 - i] = v;
                        S.LF[0][16 - i] = f;
                    } else if (i == 16) {
                        S.L[0][0] = S.T[0][0] = v;
                        S.LF[0][0] = S.TF[0][0] = f;
                    } else {
                        S.T[0][i - 16] = v;
                        S.TF[0][i - 16] = f;
                    }
                }
                // DC: luma L[1..8] (i 8..15) + T[1..8] (i 17..24); chroma c: L[1..4] (q 4..7), T[1..4] (q 9..12)
                dcl = wsum((i >= 8 && i <= 15) || (i >= 17 && i <= 24) ? v : 0);
                const int qc = i - 33, qq = qc - 17;
                dcc0 = wsum(i >= 33 && ((qc >= 4 && qc <= 7) || (qc >= 9 && qc <= 12)) ? v : 0);
                dcc1 = wsum(i >= 50 && ((qq >= 4 && qq <= 7) || (qq >= 9 && qq <= 12)) ? v : 0);
            }
        }
        dcl = (dcl + 8) >> 4;
        dcc0 = (dcc0 + 4) >> 3;
        dcc1 = (dcc1 + 4) >> 3;
        wave_lds_sync();
        // ---- prediction and residual
        const int pl = pred_sample(mode, 3, true, S.L[0], S.T[0], S.LF[0], S.TF[0], dcl, lx, ly);
        const int ol = (by + ly) * 16 + bx + lx;
        t.res[lane] = (int16_t)((int)src[ol] - pl);
        int pc = 0, oc = 0;
        if (cl) {
            pc = pred_sample(mode, 2, false, S.L[1 + comp], S.T[1 + comp], S.L[1 + comp], S.T[1 + comp],
                             comp ? dcc1 : dcc0, cx, cy);
            oc = 256 + comp * 64 + (cby + cy) * 8 + cbx + cx;
            t.res[64 + comp * 16 + cy * 4 + cx] = (int16_t)((int)src[oc] - pc);
        }
        wave_lds_sync();
        // ---- forward stage 1 (rows): aT[k][y]
        aT[lx * 8 + ly] = (int16_t)((dot8(M.t8 + lx * 8, t.res + ly * 8) + 2) >> 2);
        if (cl) aT[64 + comp * 16 + cx * 4 + cy] = (int16_t)((dot4(M.t4 + cx * 4, t.res + 64 + comp * 16 + cy * 4) + 1) >> 1);
        wave_lds_sync();
        // ---- forward stage 2 (columns) + quantisation: lane (k2 = ly, k = lx)
        {
            const int l = quant_coef((dot8(M.t8 + ly * 8, aT + lx * 8) + 256) >> 9, qp, 3, true);
            const int si = scan_index_s(3, scan, lx, ly);
            coef[64 * k + si] = (int16_t)l;
            lv[64 * k + si] = (int16_t)l;
            bT[lx * 8 + ly] = (int16_t)dequant_coef(l, qp, 3);
        }
        if (cl) {
            const int l = quant_coef((dot4(M.t4 + cy * 4, aT + 64 + comp * 16 + cx * 4) + 128) >> 8, qpc, 2, true);
            const int si = 256 + 64 * comp + 16 * k + scan_index_s(2, scan, cx, cy);
            coef[si] = (int16_t)l;
            lv[si] = (int16_t)l;
            bT[64 + comp * 16 + cx * 4 + cy] = (int16_t)dequant_coef(l, qpc, 2);
        }
        wave_lds_sync();
        // ---- inverse stage 1 (columns): a16[y][x]
        aT[ly * 8 + lx] = (int16_t)clip16((dot8(M.tt8 + ly * 8, bT + lx * 8) + 64) >> 7);
        if (cl) aT[64 + comp * 16 + cy * 4 + cx] = (int16_t)clip16((dot4(M.tt4 + cy * 4, bT + 64 + comp * 16 + cx * 4) + 64) >> 7);
        wave_lds_sync();
        // ---- inverse stage 2 (rows) + reconstruction
        {
            const int v = clip255(pl + ((dot8(M.tt8 + lx * 8, aT + ly * 8) + 2048) >> 12));
            const int e = (int)src[ol] - v;
            sse_y += (x0 + bx + lx < disp_w && y0 + by + ly < disp_h) ? e * e : 0;
            t.pred[ol] = (uint8_t)v;
            rec_y[(size_t)(y0 + by + ly) * pitch + x0 + bx + lx] = (uint8_t)v;
        }
        if (cl) {
            const int v = clip255(pc + ((dot4(M.tt4 + cx * 4, aT + 64 + comp * 16 + cy * 4) + 2048) >> 12));
            const int e = (int)src[oc] - v;
            const int xc = x0 / 2 + cbx + cx, yc = y0 / 2 + cby + cy;
            sse_c += (2 * xc < disp_w && 2 * yc < disp_h) ? e * e : 0;
            t.pred[oc] = (uint8_t)v;
            rec_uv[(size_t)yc * pitch + 2 * xc + comp] = (uint8_t)v;
        }
        wave_lds_sync();
    }
    SplitIntraResult out;
    out.sse[0] = wsum(sse_y);
    out.sse[1] = wsum(comp == 0 && cl ? sse_c : 0);
    out.sse[2] = wsum(comp == 1 && cl ? sse_c : 0);
    // cu_bits_est (split, no 4x4 luma): per TU 4 + 2 floor(log2 |l|) per level, + 4 if coded, else 1
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int l = lv[64 * j + lane], a = l < 0 ? -l : l;
        const int b = a ? 4 + 2 * (31 - __builtin_clz((uint32_t)a)) : 0;
        if (j < 4) {
            const int sum = wsum(b);
            bits += (uint32_t)(__ballot(a != 0) ? sum + 4 : 1);
        } else {  // four 4x4 chroma TUs of 16 levels
            const int sum = gsum<16>(b);
            const uint64_t any = __ballot(a != 0);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bits += (uint32_t)(((any >> (16 * q)) & 0xffffu) ? __builtin_amdgcn_readlane(sum, 16 * q) + 4 : 1);
        }
    }
    out.bits = bits;
    return out;
}

__global__ __launch_bounds__(64 * kMaxSliceRows) void k_hevc_intra(Geometry g, const HevcFrameState* __restrict__ fs,
                                                      const uint8_t* __restrict__ src_y,
                                                      const uint8_t* __restrict__ src_uv, CuInfo* __restrict__ cus,
                                                      int16_t* __restrict__ coef, const uint8_t* __restrict__ imode,
                                                      uint8_t* __restrict__ qp_coded) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    // dynamic LDS: per row of the slice, the bottom luma row and bottom chroma (NV12) row
    extern __shared__ uint8_t bottom[];
    __shared__ Mats M;
    __shared__ TuBuf tb[kMaxSliceRows];
    __shared__ IntraRefs rf[kMaxSliceRows];
    __shared__ uint8_t leftc[kMaxSliceRows][32];  // right column of the wave's previous CU: 16 Y, 8 Cb, 8 Cr
    __shared__ SplitRefs srf[kMaxSliceRows];          // split units: TU references (split_intra_code)
    __shared__ alignas(16) uint8_t srcs[kMaxSliceRows][384];  // split units: the unit's source (t.pred layout)
    // units of each row finished: its bottom lines are in LDS up to there (the row below waits on it)
    __shared__ int prog[kMaxSliceRows];
    fill_mats(M);
    if (threadIdx.x < kMaxSliceRows) prog[threadIdx.x] = 0;
    __syncthreads();  // the only workgroup barrier: from here every wave runs its row alone
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sr = fs->slice_rows;
    const int row = wave;  // one wave per unit row of the slice
    // slice blockIdx.x: segment seg of CTB row band blockIdx.x / split (unit columns [xb, xe))
    const int seg_w = fs->i_seg_w, split = (g.mb_w + seg_w - 1) / seg_w;
    const int seg = (int)blockIdx.x % split, xb = seg * seg_w, xe = min(g.mb_w, xb + seg_w);
    const int y = ((int)blockIdx.x / split) * sr + row;  // CTU row of this wave
    if (row >= sr || y >= g.mb_h) return;  // wave-uniform; no workgroup barrier below, nobody waits on it
    const int qp = fs->qp;
    const int qpc = chroma_qp(qp, fs->chroma_qp_offset);
    const int cw = g.coded_w;
    uint8_t* bot_y = bottom + (size_t)row * 2 * cw;
    uint8_t* bot_c = bot_y + cw;
    const uint8_t* up_y = bottom + (size_t)(row - 1) * 2 * cw;  // row above (same slice), valid if row > 0
    const uint8_t* up_c = up_y + cw;
    TuBuf& t = tb[wave];
    IntraRefs& R = rf[wave];
    unsigned long long acc[3] = {0, 0, 0};
    // this lane's source samples of the CTU, loaded a unit ahead (off the critical path):
    // luma row lane / 4, columns 4 (lane % 4) .. +3; chroma row lane / 8, Cb/Cr pair lane % 8
    auto load_src = [&](int xx, uint32_t& ly, uint32_t& lc) {
        if (xx >= xe) return;
        const int r = lane >> 2, cb = (lane & 3) * 4, rc = lane >> 3, cc = lane & 7;
        ly = *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y * 16 + r) * g.pitch + xx * 16 + cb);
        lc = *reinterpret_cast<const uint16_t*>(src_uv + (size_t)(y * 8 + rc) * g.pitch + xx * 16 + 2 * cc);
    };
    uint32_t nsy = 0, nsc = 0;
    load_src(xb, nsy, nsc);
    // The rows of a slice form a wavefront through the progress counters alone (as k_intra_wave):
    // unit x of row r needs units x - 1 .. x + 1 of row r - 1 (corner, top, top-right), so a split
    // unit (four serial TU chains) delays only the rows below it, and only when they catch up.
    for (int x = xb; x < xe; ++x) {
        const int x0 = x * 16, y0 = y * 16;
        const uint32_t sy4 = nsy, sc2 = nsc;
        load_src(x + 1, nsy, nsc);
        // availability in the decoder's z order: a CTB's last unit has no above-right; its first
        // unit's below-left (the left CTB's last unit) is available there but not reconstructed yet
        // by this raster wavefront: k_hevc_intra_modes gave that unit a mode that never reads it
        const int z = ((y & 1) << 1) | (x & 1);
        const bool al = x > xb, at = row > 0, atr = at && x + 1 < xe && z != 3, ac = at && x > xb;
        if (at) {
            const int need = (atr ? x + 2 : x + 1) - xb;
            while (__hip_atomic_load(&prog[row - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
                __builtin_amdgcn_s_sleep(1);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
        }
        // ---- gather neighbour samples (left from LDS, above from the upper wave's bottom row)
        if (lane < 16) {
            R.lpx[lane] = al ? leftc[wave][lane] : 0;
            R.tpx[lane] = at ? up_y[x0 + lane] : 0;
            R.trx[lane] = atr ? up_y[x0 + 16 + lane] : 0;
        } else if (lane < 32) {
            const int k = lane - 16, comp = k >> 3, q = k & 7;
            R.lc[comp][q] = al ? leftc[wave][16 + comp * 8 + q] : 0;
            R.tc[comp][q] = at ? up_c[x0 + 2 * q + comp] : 0;
            R.trc[comp][q] = atr ? up_c[x0 + 16 + 2 * q + comp] : 0;
        } else if (lane == 32) {
            R.corner = ac ? up_y[x0 - 1] : 0;
            R.corner_c[0] = ac ? up_c[x0 - 2] : 0;
            R.corner_c[1] = ac ? up_c[x0 - 1] : 0;
        }
        wave_lds_sync();
        // ---- the mode (and the split) decided open-loop by k_hevc_intra_modes
        const int im = (int)imode[y * g.mb_w + x];  // (wave-uniform)
        const int mode = im & (kIntraSplitFlag - 1);
        const bool split = (im & kIntraSplitFlag) != 0;
        const int i = y * g.mb_w + x;
        if (split) {
            // four 8x8 TUs, each predicted from the reconstruction of the TUs before it
            uint8_t* sb = srcs[wave];
            {
                const int r = lane >> 2, cb = (lane & 3) * 4, rc = lane >> 3, cc = lane & 7;
                *reinterpret_cast<uint32_t*>(sb + r * 16 + cb) = sy4;
                sb[256 + rc * 8 + cc] = (uint8_t)(sc2 & 0xff);
                sb[256 + 64 + rc * 8 + cc] = (uint8_t)(sc2 >> 8);
            }
            wave_lds_sync();
            int16_t* lvs = reinterpret_cast<int16_t*>(t.b) + 384;
            const SplitIntraResult sres =
                split_intra_code(t, srf[wave], R, M, sb, lvs, mode, qp, qpc, al, ac, at, atr, coef + (size_t)i * kCoefPerCu,
                                 fs->rec_y, fs->rec_uv, g.pitch, x0, y0, g.width, g.height);
            acc[0] += (unsigned)sres.sse[0];
            acc[1] += (unsigned)sres.sse[1];
            acc[2] += (unsigned)sres.sse[2];
            const SplitSummary ss = split_summary_wave(lvs, lane, 0);
            if (lane == 0) {
                CuInfo c{};
                c.type = kCuIntra;
                c.intra_mode = (uint8_t)mode;
                c.qp = (uint8_t)qp;
                c.tu_split = 2;
                ss.apply(c);
                c.ct = 1;
                set_est_bytes(c, sres.bits);
                cus[i] = c;
                qp_coded[i] = c.cbf ? c.qp : (uint8_t)255;
            }
        } else {
            // ---- reference substitution (8.4.4.2.2) for every sample at once, then the planar
            // filter and DC sums; the same values as intra_refs() + the lane-serial loops this
            // replaced (their availability/pointer lambdas lived in scratch: two dependent memory
            // round trips per reference sample on the wavefront's critical path)
            const int avl = (al ? 2 : 0) | (ac ? 4 : 0) | (at ? 8 : 0) | (atr ? 16 : 0);  // no bottom-left
            for (int q = lane; q <= 64; q += 64) {
                const int v = ref_subst(q, 16, avl, R.lpx, R.tpx, R.trx, R.corner);
                if (q < 32) R.L[32 - q] = v;
                else if (q == 32) R.L[0] = R.T[0] = v;
                else R.T[q - 32] = v;
            }
            for (int k = lane; k < 66; k += 64) {
                const int comp = k >= 33 ? 1 : 0, q = k - 33 * comp;
                const int v = ref_subst(q, 8, avl, R.lc[comp], R.tc[comp], R.trc[comp], R.corner_c[comp]);
                if (q < 16) R.Lc[comp][16 - q] = v;
                else if (q == 16) R.Lc[comp][0] = R.Tc[comp][0] = v;
                else R.Tc[comp][q - 16] = v;
            }
            wave_lds_sync();
            if (lane <= 32) {
                const int k = lane;
                if (k == 0) {
                    R.LF[0] = R.TF[0] = (R.L[1] + 2 * R.L[0] + R.T[1] + 2) >> 2;
                } else if (k == 32) {
                    R.LF[32] = R.L[32];
                    R.TF[32] = R.T[32];
                } else {
                    R.LF[k] = (R.L[k + 1] + 2 * R.L[k] + R.L[k - 1] + 2) >> 2;
                    R.TF[k] = (R.T[k + 1] + 2 * R.T[k] + R.T[k - 1] + 2) >> 2;
                }
            }
            const int sl = lane < 16 ? R.L[1 + lane] + R.T[1 + lane] : 0;
            const int c0 = (lane >= 16 && lane < 24) ? R.Lc[0][lane - 15] + R.Tc[0][lane - 15] : 0;
            const int c1 = (lane >= 24 && lane < 32) ? R.Lc[1][lane - 23] + R.Tc[1][lane - 23] : 0;
            const int dcl = (wsum(sl) + 16) >> 5, dc0 = (wsum(c0) + 8) >> 4, dc1 = (wsum(c1) + 8) >> 4;
            wave_lds_sync();
            const int r = lane >> 2, cb = (lane & 3) * 4;
            for (int j = 0; j < 4; ++j) {
                const int p = pred_sample(mode, 4, true, R.L, R.T, R.LF, R.TF, dcl, cb + j, r);
                t.pred[r * 16 + cb + j] = (uint8_t)p;
                t.res[r * 16 + cb + j] = (int16_t)((int)((sy4 >> (8 * j)) & 0xff) - p);
            }
            const int rc = lane >> 3, cc = lane & 7;
            for (int comp = 0; comp < 2; ++comp) {
                const int p = pred_sample(mode, 3, false, R.Lc[comp], R.Tc[comp], R.Lc[comp], R.Tc[comp],
                                          comp ? dc1 : dc0, cc, rc);
                t.pred[256 + comp * 64 + rc * 8 + cc] = (uint8_t)p;
                t.res[256 + comp * 64 + rc * 8 + cc] = (int16_t)((int)((sc2 >> (8 * comp)) & 0xff) - p);
            }
            wave_lds_sync();
            const TuResult res = code_tus<false>(t, M, qp, qpc, true, true, coef + (size_t)i * kCoefPerCu, fs->rec_y,
                                                 g.pitch, fs->rec_uv, x0, y0, g.width, g.height);
            acc[0] += (unsigned)res.sse[0];
            acc[1] += (unsigned)res.sse[1];
            acc[2] += (unsigned)res.sse[2];
            if (lane == 0) {
                CuInfo c{};
                c.type = kCuIntra;
                c.intra_mode = (uint8_t)mode;
                c.qp = (uint8_t)qp;
                c.mvx = c.mvy = c.mvdx = c.mvdy = 0;
                c.mvp_idx = 0;
                fill_cu(c, res);
                c.ct = 1;
                set_est_bytes(c, res.bits);
                cus[i] = c;
                // (no slice cost: I pictures use fixed CTB-row slices)
                qp_coded[i] = c.cbf ? c.qp : (uint8_t)255;
            }
        }
        wave_lds_sync();
        // reconstruction edges (kept in t.pred): right column -> left neighbour of this row's next
        // unit, bottom rows -> the row below, then publish the unit
        if (lane < 16) {
            leftc[wave][lane] = t.pred[lane * 16 + 15];
            bot_y[x0 + lane] = t.pred[15 * 16 + lane];
            bot_c[x0 + lane] = t.pred[256 + (lane & 1) * 64 + 7 * 8 + (lane >> 1)];
        } else if (lane < 32) {
            const int k = lane - 16, comp = k >> 3, q = k & 7;
            leftc[wave][16 + comp * 8 + q] = t.pred[256 + comp * 64 + q * 8 + 7];
        }
        wave_lds_sync();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // LDS completes the line stores before the counter
        if (lane == 0) __hip_atomic_store(&prog[row], x - xb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (lane < 3)  // wave sums (identical in every lane)
        fs->sse_part[lane * h264::kSsePartStride + y * split + seg] = lane == 0 ? acc[0] : (lane == 1 ? acc[1] : acc[2]);
}

// ------------------------------------------------------------------ slice layout
// One 1024-thread workgroup.  I pictures: fixed slices of slice_rows CTU rows.  P pictures:
// cost-balanced raster runs (hevc_core.h plan_*): each thread owns a chunk of CUs; a wave-level
// prefix sum of the chunk costs gives every CU its exclusive cost prefix, and the slice id
// floor(prefix * S / total) is tracked against the next slice's threshold ceil(s * total / S), so
// a 64-bit division happens per slice start rather than per CU (that division loop cost ~60 us at
// 4K).  Starts are compacted by a second prefix sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wtot, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
    uint32_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (int w = 0; w < nw; ++w) {
        before += w < wave ? wtot[w] : 0u;
        all += wtot[w];
    }
    __syncthreads();
    *total = all;
    return before + incl - v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}
// Scans over per-CU arrays run in tiles of 1024 threads x 4 consecutive CUs (arrays padded with
// zeros to a whole tile: HevcDeviceBuffers).
constexpr int kScanTile = 4096;
constexpr int kMaxScanTiles = 64;
__device__ __forceinline__ uint4 ld4(const uint32_t* p, int i) { return *reinterpret_cast<const uint4*>(p + i); }

// Tile prefixes of a per-CU array (tiles of kScanTile CUs, 4 per thread with one 16-byte load,
// arrays zero-padded to whole tiles), computed by EVERY workgroup of a one-workgroup-per-tile
// launch: the per-wave tile totals (wave_tot[t][w]) and the tiles' exclusive prefixes (tile_pre[t]);
// returns the array total.  Re-reading the whole array per workgroup is a few 16-byte loads per
// thread from L2 -- cheaper than a chained hand-off between the tiles' workgroups.
__device__ __forceinline__ uint32_t tile_prefixes(const uint32_t* __restrict__ a, int ncu, uint32_t (*wave_tot)[16],
                                                  uint32_t* tile_pre, uint32_t* total_sh) {
    const int tid = threadIdx.x, wv = tid >> 6, nwv = (int)blockDim.x >> 6;
    int nt = 0;
#pragma unroll 4
    for (int base = 0; base < ncu; base += kScanTile) {
        const uint4 v = ld4(a, base + 4 * tid);
        uint32_t w = v.x + v.y + v.z + v.w;
        for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
        if ((tid & 63) == 0) wave_tot[nt][wv] = w;
        ++nt;
    }
    __syncthreads();
    if (tid < 64) {  // one wave: tile totals and their exclusive prefix (nt <= kMaxScanTiles = 64)
        uint32_t sum = 0;
        if (tid < nt)
            for (int w = 0; w < nwv; ++w) sum += wave_tot[tid][w];
        const uint32_t incl = wave_incl_scan(sum);
        if (tid < nt) tile_pre[tid] = incl - sum;
        if (tid == 63) *total_sh = incl;
    }
    __syncthreads();
    return *total_sh;
}
// exclusive prefix of this thread's first CU in tile t (after tile_prefixes)
__device__ __forceinline__ uint32_t tile_thread_prefix(const uint32_t (*wave_tot)[16], const uint32_t* tile_pre, int t,
                                                       uint32_t sum4) {
    const int wv = threadIdx.x >> 6;
    uint32_t before = tile_pre[t];
    for (int w = 0; w < wv; ++w) before += wave_tot[t][w];
    return before + wave_incl_scan(sum4) - sum4;
}

// Slice layout, one workgroup per scan tile.  P pictures: cost-balanced raster runs -- a CTB's
// slice id is plan_slice_of of its cost prefix, a slice starts where the id changes, and a slice's
// rank counts the starts before it: a CTB heavier than the slice spacing skips ids, so ranks are
// compacted (every workgroup counts the starts of the tiles before its own -- a block reduction per
// earlier tile, cheaper than chaining the workgroups).  (Until round 5 the spacing was kept above
// the largest possible CTB cost so that ids were ranks; with CTB32 that cost is 4,504 and held a 4K
// P picture to ~107 slices of the level's 200: the slowest CABAC substream 870 us.)
__global__ __launch_bounds__(1024) void k_hevc_layout(const HevcFrameState* __restrict__ fs,
                                                       const uint32_t* __restrict__ cost, int ncu, int ctb_w,
                                                       int max_slices, int slice_cost, int* __restrict__ slice_first,
                                                       int* __restrict__ slice_of_cu, uint32_t* __restrict__ nslices) {
    const int tid = threadIdx.x, t = blockIdx.x;
    if (t == 0)
        for (int k = tid; k < kSseSlots * kSseSlotWords; k += blockDim.x) fs->sse_tot[k] = 0ull;  // k_hevc_sao adds into these next
    if (fs->idr || fs->wpp) {  // I: fixed row slices; P with WPP: slices of wpp_rows rows (a substream per row)
        const int rows = ncu / ctb_w;
        const int sr = fs->idr ? fs->slice_rows / 2 : fs->wpp_rows;  // (slice_rows counts 16x16-unit rows)
        const int S = fs->idr ? fs->num_slices : (rows + sr - 1) / sr;
        // I: segments of segc CTBs (split per row band, i_seg_range); WPP: whole rows
        const int segc = fs->idr ? fs->i_seg_w / 2 : ctb_w, split = (ctb_w + segc - 1) / segc;
        const int stride = (int)(gridDim.x * blockDim.x);
        for (int k = t * (int)blockDim.x + tid; k < S; k += stride)
            slice_first[k] = (k / split) * sr * ctb_w + (k % split) * segc;
        for (int i = t * (int)blockDim.x + tid; i < ncu; i += stride)
            slice_of_cu[i] = ((i / ctb_w) / sr) * split + (i % ctb_w) / segc;
        if (t == 0 && tid == 0) *nslices = (uint32_t)S;
        return;
    }
    __shared__ uint32_t tile_pre[kMaxScanTiles];
    __shared__ uint32_t wave_tot[kMaxScanTiles][16];
    __shared__ uint32_t total_sh;
    __shared__ uint32_t wave_starts[16];
    const uint32_t total = tile_prefixes(cost, ncu, wave_tot, tile_pre, &total_sh);
    const int S = plan_num_slices(total, max_slices, (uint32_t)slice_cost);
    const int wv = tid >> 6, nwv = (int)blockDim.x >> 6;
    uint32_t base = 0;  // slice starts in the tiles before this one
    for (int tt = 0; tt <= t; ++tt) {
        const int i0 = tt * kScanTile + 4 * tid;
        const uint4 v = ld4(cost, i0);
        const uint32_t c4[4] = {v.x, v.y, v.z, v.w};
        uint64_t pre = tile_thread_prefix(wave_tot, tile_pre, tt, v.x + v.y + v.z + v.w);
        int id[4];
        uint32_t st = 0;  // bit e: CTB i0 + e starts a slice
        int prev = i0 > 0 && i0 < ncu ? plan_slice_of(pre - cost[i0 - 1], total, S) : -1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            id[e] = plan_slice_of(pre, total, S);
            if (i0 + e < ncu && id[e] != prev) st |= 1u << e;
            prev = id[e];
            pre += c4[e];
        }
        const uint32_t cnt = (uint32_t)__popc(st);
        const uint32_t incl = wave_incl_scan(cnt);
        if ((tid & 63) == 63) wave_starts[wv] = incl;
        __syncthreads();
        uint32_t before = base, tile_cnt = 0;
        for (int w = 0; w < nwv; ++w) {
            if (w < wv) before += wave_starts[w];
            tile_cnt += wave_starts[w];
        }
        __syncthreads();
        if (tt < t) {
            base += tile_cnt;
            continue;
        }
        int r = (int)(before + incl - cnt) - 1;  // rank of the slice holding the CTB before i0
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (i0 + e >= ncu) break;
            if ((st >> e) & 1u) {
                ++r;
                slice_first[r] = i0 + e;
            }
            slice_of_cu[i0 + e] = r;
        }
        if (tid == 0 && (t + 1) * kScanTile >= ncu) *nslices = base + tile_cnt;  // the last tile's workgroup
    }
}

// Skip / merge / AMVP of the units of a P picture against their slice's neighbours and the coding
// tree of every CTB (hevc_core.h decide_ctb): one thread per CTB.
__global__ __launch_bounds__(256) void k_hevc_decide(Geometry g, const h264::MbInfo* __restrict__ mbs,
                                                      const int* __restrict__ slice_first,
                                                      const int* __restrict__ slice_of_ctb, CuInfo* __restrict__ cus) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int cw = ctb_cols(g.mb_w);
    if (c >= cw * ctb_rows(g.mb_h)) return;
    constexpr int kStride = sizeof(h264::MbInfo) / sizeof(int16_t);
    const int x0 = 2 * (c % cw), y0 = 2 * (c / cw);
    CuInfo u[4];
    bool in[4];
#pragma unroll
    for (int z = 0; z < 4; ++z) {
        const int x = x0 + (z & 1), y = y0 + (z >> 1);
        in[z] = x < g.mb_w && y < g.mb_h;
        if (in[z]) u[z] = cus[y * g.mb_w + x];
    }
    decide_ctb(u, in, &mbs[0].mvx, kStride, x0, y0, g.mb_w, g.mb_h, slice_first[slice_of_ctb[c]]);
#pragma unroll
    for (int z = 0; z < 4; ++z)
        if (in[z]) cus[(y0 + (z >> 1)) * g.mb_w + x0 + (z & 1)] = u[z];
}

__device__ __forceinline__ CuInfo load_cu(const CuInfo* cus, int i) {
    // kCuWords dwords (CuInfo is 24 bytes, 4-byte aligned in the array) -> wave-uniform values
    const uint32_t* p = reinterpret_cast<const uint32_t*>(cus) + (size_t)i * kCuWords;
    uint32_t w[kCuWords];
    for (int q = 0; q < kCuWords; ++q) w[q] = (uint32_t)__builtin_amdgcn_readfirstlane((int)p[q]);
    CuInfo c{};
    __builtin_memcpy(&c, w, sizeof c);
    return c;
}

// ------------------------------------------------------------------ CABAC
// Two phases (hevc_core.h "bin tokens").  Binarisation is a pure function of a CTU, its
// neighbours' descriptors and its QP predictor (qpy of the previous CTU in the slice), so
// k_hevc_bins binarises every CTU of the picture at once -- one wave per CTU, one lane per part
// (hevc_core.h for_each_part: head, split-child heads, TU last positions, sub-blocks) staged in
// LDS and concatenated by a wave prefix sum -- into a fixed slot of kMaxCuTokens tokens; k_hevc_tokscan / k_hevc_tokgather lay the tokens of the picture out
// densely in decoding order.  Only the arithmetic coder is serial: k_hevc_arith runs one wave per
// slice over that slice's token run -- a short loop with no syntax logic, whose coder state lives
// in SGPRs and whose 144 context states sit four to a lane in one VGPR (v_readlane /
// v_writelane), so the serial part is a few dozen scalar instructions per token and fits the
// instruction cache (the former single-phase kernel was 16 k instructions of CU syntax per wave
// and took ~0.8 us per skipped CTU: profiles/r03_cabac).
// One wave per coding position (4 per CTB, z order; positions outside the picture emit nothing).
struct CuGet {  // wave-uniform CuInfo loads for unit_syn
    const CuInfo* p;
    __device__ __forceinline__ CuInfo operator()(int u) const { return load_cu(p, u); }
};
__global__ __launch_bounds__(64) void k_hevc_bins(Geometry g, const HevcFrameState* __restrict__ fs,
                                                   const CuInfo* __restrict__ cus, const int16_t* __restrict__ coef,
                                                   const uint32_t* __restrict__ sao,
                                                   const int* __restrict__ slice_first,
                                                   const int* __restrict__ slice_of_ctb,
                                                   const uint32_t* __restrict__ nslices,
                                                   const uint8_t* __restrict__ qp_pred, uint16_t* __restrict__ tok,
                                                   uint32_t* __restrict__ ntok) {
    __shared__ uint16_t stage[64 * kPartTokens];
    const int k = blockIdx.x, lane = threadIdx.x;
    const int cw = ctb_cols(g.mb_w), nctb = cw * ctb_rows(g.mb_h);
    int x, y;
    cpos_xy(k, cw, &x, &y);
    if (x >= g.mb_w || y >= g.mb_h) {
        if (lane == 0) ntok[k] = 0;
        return;
    }
    const int i = y * g.mb_w + x, c = k >> 2;
    const int ns = (int)uni(*nslices);
    const int s = uni(slice_of_ctb[c]);
    const int first = uni(slice_first[s]);
    const int end = s + 1 < ns ? uni(slice_first[s + 1]) : nctb;
    const UnitSyn u = unit_syn(CuGet{cus}, fs->sao ? sao : nullptr, x, y, g.mb_w, g.mb_h, fs->idr != 0, first, end,
                               fs->wpp != 0, fs->depth_inter, fs->depth_intra, (int)uni((uint32_t)qp_pred[i]));
    const CuInfo cu = load_cu(cus, i);
    const CoefArray cf{coef + (size_t)i * kCoefPerCu};
    // lane p binarises part p of the unit (coding order) into its LDS run
    CtuPart mine;
    bool have = false;
    for_each_part(cu, u, cf, [&](const CtuPart& pt, int idx) {
        if (idx == lane) {
            mine = pt;
            have = true;
        }
    });
    BinRec rec;
    rec.start(stage + lane * kPartTokens, kPartTokens);
    NoCtx nc;
    if (have) binarise_part(rec, nc, mine, cu, u, cf);
    const uint32_t n = have ? min(rec.n, kPartTokens) : 0u;
    uint32_t incl = n;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    uint16_t* dst = tok + (size_t)k * kMaxCuTokens + (incl - n);
    const uint16_t* src = stage + lane * kPartTokens;
    for (uint32_t j = 0; j < n; ++j) dst[j] = src[j];
    if (lane == 63) ntok[k] = incl;
}

// Exclusive prefix of the token counts in decoding order (coding positions): off[k], off[n] = total.
// One 1024-thread workgroup per scan tile (tile_prefixes), 16-byte loads and stores.
__global__ __launch_bounds__(1024) void k_hevc_tokscan(const uint32_t* __restrict__ ntok, int ncu,
                                                        uint32_t* __restrict__ off) {
    __shared__ uint32_t tile_pre[kMaxScanTiles];
    __shared__ uint32_t wave_tot[kMaxScanTiles][16];
    __shared__ uint32_t total_sh;
    const int tid = threadIdx.x, t = blockIdx.x;
    const uint32_t total = tile_prefixes(ntok, ncu, wave_tot, tile_pre, &total_sh);
    const int i = t * kScanTile + 4 * tid;
    const uint4 v = ld4(ntok, i);
    const uint32_t pre = tile_thread_prefix(wave_tot, tile_pre, t, v.x + v.y + v.z + v.w);
    *reinterpret_cast<uint4*>(off + i) = make_uint4(pre, pre + v.x, pre + v.x + v.y, pre + v.x + v.y + v.z);
    if (t == 0 && tid == 0) off[ncu] = total;  // (the padded tail of the last tile holds the total too)
}

// One wave per CTU: copy its tokens from the fixed slot to the dense run.
__global__ __launch_bounds__(256) void k_hevc_tokgather(const uint16_t* __restrict__ tok,
                                                         const uint32_t* __restrict__ ntok,
                                                         const uint32_t* __restrict__ off, int ncu,
                                                         uint16_t* __restrict__ dense) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= ncu) return;
    const uint32_t n = ntok[i], o = off[i];
    const uint16_t* src = tok + (size_t)i * kMaxCuTokens;
    for (uint32_t t = lane; t < n; t += 64) dense[o + t] = src[t];
}

// Context states for the serial coder: lane l of `st` holds states 4l .. 4l+3 (one byte each),
// lane s of lps_row / next holds rangeTabLps[s][0..3] and transIdxLps[s].
struct PackedCtx {
    uint32_t st;
    uint32_t lps_row, next;
    int lane;
    __device__ __forceinline__ uint32_t get(int i) const {
        return ((uint32_t)__builtin_amdgcn_readlane((int)st, i >> 2) >> ((i & 3) * 8)) & 0xffu;
    }
    __device__ __forceinline__ void set(int i, uint32_t v) {
        const int sh = (i & 3) * 8;
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)st, i >> 2);
        const uint32_t nw = (w & ~(0xffu << sh)) | (v << sh);
        st = lane == (i >> 2) ? nw : st;  // v_cndmask: only the owning lane takes the new word
    }
    __device__ __forceinline__ uint32_t lps(uint32_t s, uint32_t q) const {
        return ((uint32_t)__builtin_amdgcn_readlane((int)lps_row, (int)s) >> (8 * q)) & 0xffu;
    }
    __device__ __forceinline__ uint32_t next_lps(uint32_t s) const {
        return (uint32_t)__builtin_amdgcn_readlane((int)next, (int)s);
    }
};

// Token -> arithmetic coder, written for the scalar unit: one wave issues at most one instruction
// every 4 cycles, so the per-token instruction count is the coder's speed.  The context bin is
// branch-free (both successor states formed, one selected; one renormalisation shift from the
// leading-zero count); the coder registers and the output position live in SGPRs and the bytes
// are stored by every lane (same address).  Same arithmetic as hevc_core.h CabacEnc, which
// finishes the slice (its registers are handed over).
struct LeanCoder {
    CabacEnc e;
    __device__ __forceinline__ void token(PackedCtx& ctx, uint32_t t) {
        if (!(t & 0x8000u)) {
            const uint32_t idx = t >> 1, b = t & 1u;
            if (idx != kTokTerm) {
                const uint32_t li = idx >> 2, sh = (idx & 3u) * 8u;
                const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)ctx.st, (int)li);
                const uint32_t s7 = (w >> sh) & 0xffu, ps = s7 >> 1, mps = s7 & 1u;
                const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)ctx.lps_row, (int)ps);
                const uint32_t nl = (uint32_t)__builtin_amdgcn_readlane((int)ctx.next, (int)ps);
                const uint32_t lps = (row >> (((e.range >> 6) & 3u) * 8u)) & 0xffu;
                const uint32_t rm = e.range - lps;
                const bool is_lps = b != mps;
                const uint32_t ns_lps = (nl << 1) | (mps ^ ((ps - 1u) >> 31));  // valMps flips on an LPS in state 0
                const uint32_t ns_mps = ((ps < 62u ? ps + 1u : 62u) << 1) | mps;
                const uint32_t nw = (w & ~(0xffu << sh)) | ((is_lps ? ns_lps : ns_mps) << sh);
                // one v_writelane (operands from the scalar unit; no exec-masked region)
                asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(ctx.st) : "s"(nw), "{m0}"(li));
                e.low += is_lps ? rm : 0u;
                const uint32_t r = is_lps ? lps : rm;
                const int n = __builtin_clz(r) - 23;
                e.low <<= n;
                e.range = r << n;
                e.bits_left -= n;
                if (e.bits_left < 12) e.write_out();
                return;
            }
            e.terminate((int)b);
            return;
        }
        e.bypass_bits(t & 0x7ffu, (int)((t >> 11) & 15u) + 1);
    }
};

// One wave per substream -- a slice, or with WPP a CTU row of a slice -- running its dense token
// run through the arithmetic coder.  Tokens arrive 256 at a time (8 bytes per lane, the next chunk
// in flight while this one is coded) and are read out of the chunk with v_readlane.
//
// WPP (9.3.1, 9.3.2.2): a row's wave starts from the contexts the row above had after its second
// CTU -- unless the row starts its slice or the picture is one CTU wide -- so it first waits for the
// row above to publish them: lane 0 of the publisher stores the 36 state words and then the frame's
// epoch into the row's flag with an agent-scope release store; the waiting wave spins on the flag
// with relaxed loads and, once it holds the epoch, issues an agent-scope acquire fence before
// reading the words.  Rows are dispatched in
// order and the publisher never waits on a later row, so the chain always drains; a bounded spin
// flags a timeout instead of hanging (GpuHevcEncoder::collect throws).
constexpr uint32_t kTokChunk = 256;
constexpr uint32_t kWppSpinLimit = 1u << 22;

__device__ __forceinline__ void arith_run(LeanCoder& lc, PackedCtx& ctx, const uint16_t* __restrict__ dense,
                                          uint32_t t0, uint32_t t1, int lane) {
    if (t0 >= t1) return;
    const uint32_t a0 = t0 & ~3u;  // 8-byte aligned chunk starts
    const uint2* src = reinterpret_cast<const uint2*>(dense + a0);
    uint2 cur = src[lane];
    for (uint32_t c = a0; c < t1; c += kTokChunk) {
        const uint2 nxt = c + kTokChunk < t1 ? src[(c + kTokChunk - a0) / 4 + lane] : make_uint2(0u, 0u);
        const uint32_t j0 = c < t0 ? t0 - c : 0u;
        const uint32_t j1 = t1 - c < kTokChunk ? t1 - c : kTokChunk;
        // the chunk's registers are consumed here, once: otherwise the wait for them lands inside the
        // token loop as a vmcnt(0) that also drains the prefetch and the coder's byte stores
        uint32_t cx = cur.x, cy = cur.y;
        asm volatile("" : "+v"(cx), "+v"(cy));
        // lane l holds tokens 4l .. 4l+3; whole lanes in the middle of the run, partial ones at its ends
        for (uint32_t l = j0 >> 2; l < (j1 + 3) >> 2; ++l) {
            const uint32_t wx = (uint32_t)__builtin_amdgcn_readlane((int)cx, (int)l);
            const uint32_t wy = (uint32_t)__builtin_amdgcn_readlane((int)cy, (int)l);
            const uint32_t j = 4 * l;
            if (j >= j0 && j + 4 <= j1) {
                lc.token(ctx, wx & 0xffffu);
                lc.token(ctx, wx >> 16);
                lc.token(ctx, wy & 0xffffu);
                lc.token(ctx, wy >> 16);
            } else {
#pragma unroll 1
                for (uint32_t q = 0; q < 4; ++q)
                    if (j + q >= j0 && j + q < j1) lc.token(ctx, ((q & 2) ? wy : wx) >> ((q & 1) * 16) & 0xffffu);
            }
        }
        cur = nxt;
    }
}

__global__ __launch_bounds__(64) void k_hevc_arith(Geometry g, const HevcFrameState* __restrict__ fs,
                                                    const uint16_t* __restrict__ dense,
                                                    const uint32_t* __restrict__ off,
                                                    const int* __restrict__ slice_first,
                                                    const int* __restrict__ slice_of_cu,
                                                    const uint32_t* __restrict__ nslices,
                                                    uint8_t* __restrict__ slice_data, uint32_t slice_cap,
                                                    uint32_t* __restrict__ slice_len,
                                                    unsigned long long* __restrict__ slice_clk) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    // (slices and substreams in CTBs; a CTB's tokens are coding positions 4 c .. 4 c + 3)
    const int u = blockIdx.x, lane = threadIdx.x;
    const bool wpp = fs->wpp != 0;
    const int cw = ctb_cols(g.mb_w), nctb = cw * ctb_rows(g.mb_h);
    const int nsub = wpp ? ctb_rows(g.mb_h) : (int)*nslices;
    if (u >= nsub) return;
    const unsigned long long clk0 = wall_clock64();
    int first, end;
    bool fresh = true, store = false;
    if (wpp) {
        first = u * cw;
        end = first + cw;
        const int s = slice_of_cu[first];
        fresh = first == slice_first[s] || cw < 2;
        store = cw >= 2 && end < nctb && slice_of_cu[end] == s;
    } else {
        const int ns = nsub;
        first = slice_first[u];
        end = u + 1 < ns ? slice_first[u + 1] : nctb;
    }
    const uint32_t t0 = uni(off[4 * first]), t1 = uni(off[4 * end]);
    const int qp = fs->qp;
    PackedCtx ctx;
    ctx.lps_row = (uint32_t)kLps[lane][0] | ((uint32_t)kLps[lane][1] << 8) | ((uint32_t)kLps[lane][2] << 16) |
                  ((uint32_t)kLps[lane][3] << 24);
    ctx.next = kNextLps[lane];
    ctx.lane = lane;
    const uint32_t epoch = fs->wpp_epoch;
    bool sync_ok = true;
    if (!fresh) {
        const uint32_t* flag = fs->wpp_flag + (u - 1);
        uint32_t n = 0;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (++n > kWppSpinLimit) {
                sync_ok = false;
                break;
            }
        }
        sync_ok = __builtin_amdgcn_readfirstlane(sync_ok ? 1 : 0) != 0;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // pairs with the publisher's release store
        if (!sync_ok && lane == 0) *fs->wpp_err = 1;
    }
    if (!fresh && sync_ok) {
        ctx.st = lane < kWppCtxWords ? fs->wpp_ctx[(size_t)(u - 1) * kWppCtxWords + lane] : 0u;
    } else {
        const int t = fs->idr ? 0 : 1;
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b) {
            const int j = 4 * lane + b;
            w |= (j < C_NUM ? (uint32_t)ctx_init_state(kCtxInit[t][j], qp) : 0u) << (8 * b);
        }
        ctx.st = w;
    }
    LeanCoder lc;
    lc.e.start(slice_data + (size_t)u * slice_cap, slice_cap);
    // two segments through one copy of the coder loop (the kernel stays inside the instruction
    // cache): the row's first two CTUs, the context publication (storage process after CTU 1),
    // then the rest; without a publication the first segment is empty
    const uint32_t ts = store ? uni(off[4 * (first + 2)]) : t0;
#pragma unroll 1
    for (int seg = 0; seg < 2; ++seg) {
        arith_run(lc, ctx, dense, seg ? ts : t0, seg ? t1 : ts, lane);
        if (seg == 0 && store && lane == 0) {
            uint32_t* dst = fs->wpp_ctx + (size_t)u * kWppCtxWords;
            for (int k = 0; k < kWppCtxWords; ++k) dst[k] = (uint32_t)__builtin_amdgcn_readlane((int)ctx.st, k);
            __hip_atomic_store(fs->wpp_flag + u, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    CabacEnc& e = lc.e;
    e.finish_slice();  // flush + the stop / alignment one-bit and zero bits (slice end or end of subset)
    if (lane == 0) {
        slice_len[u] = e.pos;
        slice_clk[2 * u] = clk0;  // diagnostics: this wave's span (GpuHevcEncoder::slice_timing)
        slice_clk[2 * u + 1] = wall_clock64();
    }
}

// ------------------------------------------------------------------ QP chain
// qPY_PRED / QpY of every unit (hevc_core.h slice_qp_chain): one workgroup per chain -- a slice, or
// with WPP a CTB row (the chain restarts at every row).  The threads stage 256 CTBs at a time (the
// four units' coded QP -- qpc, 255 when the unit sends no cu_qp_delta -- and the CTB's coding-tree
// depth).  A CTB none of whose units codes a QP passes the chain value through unchanged (every
// unit's prediction and QpY is the value entering it), so only the CTBs that code one are walked
// serially, by thread 0, in order; every other CTB then takes the value the last coded CTB before it
// left (a prefix count).  Cost-balanced slices make the static desktop a few long slices of skipped
// CTBs: the walk over all of them was the kernel's 56 us (profiles/r05_hevc/kernels_hevc4k_18M.txt).
__global__ __launch_bounds__(256) void k_hevc_qpy(Geometry g, const HevcFrameState* __restrict__ fs,
                                                   const CuInfo* __restrict__ cus, const uint8_t* __restrict__ qpc,
                                                   const int* __restrict__ slice_first,
                                                   const uint32_t* __restrict__ nslices,
                                                   uint8_t* __restrict__ qp_pred, uint8_t* __restrict__ qpy) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    __shared__ uint32_t q4[256], pr4[256], qy4[256];
    __shared__ uint8_t info[256];   // bits 0-3: unit z inside the picture, bit 4: CU32
    __shared__ uint16_t list[256];  // the chunk's QP-coding CTBs, in order
    __shared__ uint8_t after[256];  // the chain value each of them leaves
    __shared__ uint32_t wcnt[4];
    __shared__ int chunk_in;
    const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int cw = ctb_cols(g.mb_w), ch = ctb_rows(g.mb_h), nctb = cw * ch;
    const bool wpp = fs->wpp != 0;
    const int ns = wpp ? ch : (int)*nslices;
    if (s >= ns) return;
    const int first = wpp ? s * cw : slice_first[s];
    const int end = wpp ? first + cw : (s + 1 < ns ? slice_first[s + 1] : nctb);
    int prev = fs->qp;  // thread 0's chain state
    for (int base = first; base < end; base += 256) {
        const int c = base + tid;
        const int x0 = 2 * (c % cw), y0 = 2 * (c / cw);
        bool coded = false;
        if (c < end) {
            uint32_t w = 0, in = 0;
            for (int z = 0; z < 4; ++z) {
                const int x = x0 + (z & 1), y = y0 + (z >> 1);
                const bool inside = x < g.mb_w && y < g.mb_h;
                const uint32_t v = inside ? (uint32_t)qpc[y * g.mb_w + x] : 255u;
                w |= v << (8 * z);
                in |= inside ? 1u << z : 0u;
                coded |= v != 255u;
            }
            q4[tid] = w;
            info[tid] = (uint8_t)(in | (cus[y0 * g.mb_w + x0].ct == 0 ? 16u : 0u));
        }
        // position of this CTB among the chunk's coding CTBs (exclusive count)
        const unsigned long long bal = __ballot(coded);
        if (lane == 0) wcnt[wv] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        for (int k = 0; k < wv; ++k) before += wcnt[k];
        const uint32_t ncoded = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (coded) list[before] = (uint16_t)tid;
        __syncthreads();
        if (tid == 0) {
            chunk_in = prev;
            for (uint32_t k = 0; k < ncoded; ++k) {
                const int j = list[k];
                const uint32_t w = q4[j], f = info[j];
                uint32_t pw = 0, qw = 0;
                if (f & 16) {  // CU32: one quantization group, one QP
                    int q = prev;
                    for (int z = 0; z < 4; ++z)
                        if (((w >> (8 * z)) & 255u) != 255u) q = (int)((w >> (8 * z)) & 255u);
                    pw = (uint32_t)prev * 0x01010101u;
                    qw = (uint32_t)q * 0x01010101u;
                    prev = q;
                } else {
                    int qz[4] = {0, 0, 0, 0};
                    for (int z = 0; z < 4; ++z) {
                        if (!((f >> z) & 1)) continue;
                        const int qa = (z & 1) ? qz[z - 1] : prev, qb = (z & 2) ? qz[z - 2] : prev;
                        const int pred = (qa + qb + 1) >> 1;
                        const uint32_t v = (w >> (8 * z)) & 255u;
                        const int q = v != 255u ? (int)v : pred;
                        qz[z] = q;
                        pw |= (uint32_t)pred << (8 * z);
                        qw |= (uint32_t)q << (8 * z);
                        prev = q;
                    }
                }
                pr4[j] = pw;
                qy4[j] = qw;
                after[k] = (uint8_t)prev;
            }
        }
        __syncthreads();
        if (c < end) {
            if (!coded) {  // the value the last coding CTB before it left (or the chunk's entry value)
                const uint32_t v = before > 0 ? (uint32_t)after[before - 1] : (uint32_t)chunk_in;
                pr4[tid] = qy4[tid] = v * 0x01010101u;
            }
            for (int z = 0; z < 4; ++z) {
                const int x = x0 + (z & 1), y = y0 + (z >> 1);
                if (x >= g.mb_w || y >= g.mb_h) continue;
                qp_pred[y * g.mb_w + x] = (uint8_t)(pr4[tid] >> (8 * z));
                qpy[y * g.mb_w + x] = (uint8_t)(qy4[tid] >> (8 * z));
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ deblocking
// One thread per 4-sample segment of a CU's left (dir 0) or top (dir 1) edge.  Vertical
// edges are 16 samples apart and a filter reads p3..q3 / writes p2..q2, so all segments of a
// direction are independent; the horizontal pass runs as a second launch on its output.
// Adaptive in-loop filtering (EncoderConfig::deblock 2): the picture's decision by the rule of
// h264_deblock.h (coherent motion, hysteresis; an IDR keeps the last P decision), from the
// motion-search vectors of the 16x16 units.  One workgroup per 1024 units adds its counts to
// st[1..2]; the last one (ticket st[3]) decides, st[0] keeping the decision for the next picture,
// and re-arms the counters.
__global__ __launch_bounds__(1024) void k_hevc_db_auto(Geometry g, HevcFrameState* __restrict__ fs,
                                                       const h264::MbInfo* __restrict__ mb, uint32_t* __restrict__ st) {
    __shared__ uint32_t part[2][16];
    const int n = g.mb_w * g.mb_h;
    const bool idr = fs->idr != 0;
    h264::DbAutoCounts c;
    const int i = blockIdx.x * 1024 + threadIdx.x;
    if (!idr && i < n) h264::db_auto_count_mv(&mb[0].mvx, (int)(sizeof(h264::MbInfo) / 2), g.mb_w, i, c);
    uint32_t co = c.coherent, mv = c.moving;
    for (int o = 32; o > 0; o >>= 1) {
        co += __shfl_xor(co, o, 64);
        mv += __shfl_xor(mv, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = co;
        part[1][threadIdx.x >> 6] = mv;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    co = mv = 0;
    for (int k = 0; k < 16; ++k) {
        co += part[0][k];
        mv += part[1][k];
    }
    if (co) atomicAdd(&st[1], co);
    if (mv) atomicAdd(&st[2], mv);
    __threadfence();  // the counts before the ticket
    if (atomicAdd(&st[3], 1u) != gridDim.x - 1) return;
    __threadfence();
    h264::DbAutoCounts tot;
    tot.coherent = atomicAdd(&st[1], 0u);
    tot.moving = atomicAdd(&st[2], 0u);
    bool on = st[0] != 0;
    if (!idr) {
        on = h264::db_auto_decide(tot, n, on);
        st[0] = on ? 1u : 0u;
    }
    fs->deblock_on = on ? 1 : 0;
    st[1] = 0;
    st[2] = 0;
    st[3] = 0;
}

__global__ __launch_bounds__(256) void k_hevc_deblock(Geometry g, const HevcFrameState* __restrict__ fs,
                                                      const CuInfo* __restrict__ cus, const uint8_t* __restrict__ qpy,
                                                      int dir) {
    if (!fs->deblock_on) return;  // adaptive filter: off for this picture
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int ncu = g.mb_w * g.mb_h;
    if (t >= ncu * 4) return;
    const int i = t >> 2, seg = t & 3;
    if (dir == 0 ? (i % g.mb_w) != 0 : (i / g.mb_w) != 0)
        db_edge_seg(fs->rec_y, fs->rec_uv, g.pitch, g.mb_w, cus, qpy, i, dir, seg, fs->chroma_qp_offset);
    // internal 8x8 TU edge of a split CU: 8 samples from the CU edge, disjoint from its filtering
    db_internal_seg(fs->rec_y, g.pitch, g.mb_w, cus, qpy, i, dir, seg);
}

// ------------------------------------------------------------------ sample adaptive offset
// One wave per CTB (4 per workgroup), after deblocking: statistics of the deblocked picture
// (fs->rec_y / rec_uv) against the source, the per-CTB decision of hevc_core.h (sao_eval_comp /
// sao_combine, spread over the lanes: 48 edge (component, class, category) offsets, 96 band
// offsets, 96 band windows), then the offsets applied into fs->sao_y / sao_uv -- a separate
// picture, so every CTB reads deblocked neighbours -- with the final distortion over the display
// area accumulated on the way (one partial per workgroup, k_hevc_pack sums them).
// Lane mapping: luma row lane >> 2, columns 4 (lane & 3) .. + 3; chroma sample (lane & 7,
// lane >> 3) of both components.  Statistics are packed (count << 20) + sum (|sum| <= 255 * 256
// < 2^19, count <= 256).
struct SaoWave {
    int32_t eo[3][16];  // [comp][class * 4 + category - 1], packed
    int32_t bo[3][32];  // [comp][band], packed
    int32_t jeo[3][16];
    int32_t oeo[3][16];
    int32_t jb[3][32];
    int32_t ob[3][32];
    SaoCompChoice ch[3];
    uint32_t w[3];
};
typedef __attribute__((address_space(1))) uint32_t sao_gu32;
typedef __attribute__((address_space(1))) uint16_t sao_gu16;
typedef __attribute__((address_space(1))) uint8_t sao_gu8;
__device__ __forceinline__ int sao_unpack_sum(int v) { return (int)((uint32_t)v << 12) >> 12; }
__device__ __forceinline__ int sao_unpack_cnt(int v) { return (v - sao_unpack_sum(v)) >> 20; }

// 3x3 neighbourhood rows of the lane's luma samples: n[row][0..5] = columns c0 - 1 .. c0 + 4
// (-1 outside the picture); the middle four come from one dword load.
__device__ __forceinline__ void sao_luma_window(const uint8_t* p, int pitch, int W, int H, int x, int y, int (*n)[6]) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int yy = y + j - 1;
        if (yy < 0 || yy >= H) {
#pragma unroll
            for (int q = 0; q < 6; ++q) n[j][q] = -1;
            continue;
        }
        const sao_gu8* row = (const sao_gu8*)(p + (size_t)yy * pitch);
        const uint32_t mid = *(const sao_gu32*)(row + x);
        n[j][0] = x > 0 ? (int)row[x - 1] : -1;
#pragma unroll
        for (int q = 0; q < 4; ++q) n[j][1 + q] = (int)((mid >> (8 * q)) & 255);
        n[j][5] = x + 4 < W ? (int)row[x + 4] : -1;
    }
}
// 3x3 neighbourhood of chroma sample (x, y) for both components (interleaved NV12 pairs)
__device__ __forceinline__ void sao_chroma_window(const uint8_t* p, int pitch, int W, int H, int x, int y,
                                                  int (*u)[3], int (*v)[3]) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int yy = y + j - 1;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int xx = x + q - 1;
            const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
            const uint32_t pr = in ? *(const sao_gu16*)(p + (size_t)yy * pitch + 2 * xx) : 0xffffffffu;
            u[j][q] = in ? (int)(pr & 255) : -1;
            v[j][q] = in ? (int)(pr >> 8) : -1;
        }
    }
}
// edge category of the centre of a 3x3 neighbourhood for class k (0 when a neighbour is outside)
template <int K>
__device__ __forceinline__ int sao_cat3(const int (*n)[3]) {
    const int a = n[1 + kSaoDy[K][0]][1 + kSaoDx[K][0]], b = n[1 + kSaoDy[K][1]][1 + kSaoDx[K][1]];
    return (a < 0 || b < 0) ? 0 : sao_edge_cat(n[1][1], a, b);
}
// the four class categories of the centre of n, 3 bits each (class k at bits 3k..3k+2)
__device__ __forceinline__ uint32_t sao_cats(const int (*n)[3]) {
    return (uint32_t)sao_cat3<0>(n) | ((uint32_t)sao_cat3<1>(n) << 3) | ((uint32_t)sao_cat3<2>(n) << 6) |
           ((uint32_t)sao_cat3<3>(n) << 9);
}
__device__ __forceinline__ void sao_acc(int* e, int d, uint32_t cats) {
    const int v = (1 << 20) + d;
    const int c0 = (int)(cats & 7), c1 = (int)((cats >> 3) & 7), c2 = (int)((cats >> 6) & 7), c3 = (int)((cats >> 9) & 7);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        e[q] += c0 == q + 1 ? v : 0;
        e[4 + q] += c1 == q + 1 ? v : 0;
        e[8 + q] += c2 == q + 1 ? v : 0;
        e[12 + q] += c3 == q + 1 ? v : 0;
    }
}
// Sum of 16 per-lane values over the wave in 17 shuffles: four halving exchanges (xor 32, 16,
// 8, 4) leave value (lane >> 2) & 15 summed over 16 lanes, two more steps finish the sum;
// lanes with (lane & 3) == 0 return value index (lane >> 2) & 15.
__device__ __forceinline__ int sao_reduce16(int* v, int lane) {
#pragma unroll
    for (int h = 8, bit = 32; h >= 1; h >>= 1, bit >>= 1) {
        // an opaque all-ones/zero mask: a plain `hi ? v[j] : v[h + j]` is folded into a
        // dynamically indexed v[] (16-way compare/select chains, ~2,700 VALU per wave)
        int m = (lane & bit) != 0 ? -1 : 0;
        asm volatile("" : "+v"(m));
#pragma unroll
        for (int j = 0; j < h; ++j) {
            const int a = v[j], b = v[h + j];
            const int send = (a & m) | (b & ~m);
            const int keep = (b & m) | (a & ~m);
            v[j] = keep + __shfl_xor(send, bit, 64);
        }
    }
    int t = v[0];
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    return t;
}

// Each wave works on its own CTB: the phases only need the wave's own LDS writes visible
// (LDS operations of a wave complete in order), not a workgroup barrier.
__device__ __forceinline__ void sao_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void k_hevc_sao(Geometry g, const HevcFrameState* __restrict__ fs,
                                                   const uint8_t* __restrict__ src_y, const uint8_t* __restrict__ src_uv,
                                                   const CuInfo* __restrict__ cus, uint32_t* __restrict__ prm) {
    __shared__ SaoWave sw[4];
    __shared__ unsigned long long part[4][4];
    // one workgroup per 32x32 CTB, wave z = its 16x16 unit in z order: every wave gathers its unit's
    // statistics, then every wave decides from the CTB's sums (the same words in each) and applies
    // the offsets to its own unit
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bid = blockIdx.x, cw = ctb_cols(g.mb_w);
    const int ux = 2 * (bid % cw) + (wave & 1), uy = 2 * (bid / cw) + (wave >> 1);
    const bool valid = ux < g.mb_w && uy < g.mb_h;
    const int i = valid ? uy * g.mb_w + ux : 0;
    const int x0 = valid ? ux * kCtb : 0, y0 = valid ? uy * kCtb : 0;
    SaoWave& S = sw[wave];
    const uint8_t* ry = fs->rec_y;
    const uint8_t* ruv = fs->rec_uv;
    const int W = g.coded_w, H = g.coded_h, Wc = W / 2, Hc = H / 2;
    for (int k = lane; k < 96; k += 64) (&S.bo[0][0])[k] = 0;
    if (lane < 48) (&S.eo[0][0])[lane] = 0;
    sao_wave_sync();
    const int r = lane >> 2, c0 = (lane & 3) * 4;
    const int xc = x0 / 2 + (lane & 7), yc = y0 / 2 + (lane >> 3);
    // no residual anywhere in the CTB of a P picture (sao_keep_ctb): SAO off, the samples are only
    // copied and measured
    uint32_t any = 0;
    for (int z = 0; z < 4; ++z) {
        const int x = 2 * (bid % cw) + (z & 1), y = 2 * (bid / cw) + (z >> 1);
        if (x < g.mb_w && y < g.mb_h) any |= cus[y * g.mb_w + x].cbf;
    }
    const bool keep = sao_keep_ctb(fs->idr != 0, any);  // workgroup-uniform
    // ---- statistics (the edge categories and centre samples are kept for the apply phase)
    uint64_t cat_y = 0;
    uint32_t cen_y = 0, cat_u = 0, cat_v = 0, cen_uv = 0;
    if (keep) {
        cen_y = *(const sao_gu32*)(ry + (size_t)(y0 + r) * g.pitch + x0 + c0);
        cen_uv = *(const sao_gu16*)(ruv + (size_t)yc * g.pitch + 2 * xc);
    } else if (valid) {
        int L[3][6];
        sao_luma_window(ry, g.pitch, W, H, x0 + c0, y0 + r, L);
        const uint32_t sv = *(const sao_gu32*)(src_y + (size_t)(y0 + r) * g.pitch + x0 + c0);
        int e[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int n[3][3];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) n[a][b] = L[a][j + b];
            const int d = (int)((sv >> (8 * j)) & 255) - n[1][1];
            const uint32_t ck = sao_cats(n);
            cat_y |= (uint64_t)ck << (12 * j);  // re-used by the apply phase
            sao_acc(e, d, ck);
            atomicAdd(&S.bo[0][n[1][1] >> 3], (1 << 20) + d);
        }
        cen_y = (uint32_t)L[1][1] | ((uint32_t)L[1][2] << 8) | ((uint32_t)L[1][3] << 16) | ((uint32_t)L[1][4] << 24);
        int t = sao_reduce16(e, lane);
        if ((lane & 3) == 0) S.eo[0][(lane >> 2) & 15] = t;
        int U[3][3], V[3][3];
        sao_chroma_window(ruv, g.pitch, Wc, Hc, xc, yc, U, V);
        const uint32_t spair = *(const sao_gu16*)(src_uv + (size_t)yc * g.pitch + 2 * xc);
        const int du = (int)(spair & 255) - U[1][1], dv = (int)(spair >> 8) - V[1][1];
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = 0;
        cat_u = sao_cats(U);
        cat_v = sao_cats(V);
        cen_uv = (uint32_t)U[1][1] | ((uint32_t)V[1][1] << 8);
        sao_acc(e, du, cat_u);
        atomicAdd(&S.bo[1][U[1][1] >> 3], (1 << 20) + du);
        t = sao_reduce16(e, lane);
        if ((lane & 3) == 0) S.eo[1][(lane >> 2) & 15] = t;
#pragma unroll
        for (int q = 0; q < 16; ++q) e[q] = 0;
        sao_acc(e, dv, cat_v);
        atomicAdd(&S.bo[2][V[1][1] >> 3], (1 << 20) + dv);
        t = sao_reduce16(e, lane);
        if ((lane & 3) == 0) S.eo[2][(lane >> 2) & 15] = t;
    }
    __syncthreads();  // the CTB's four units' statistics
    // ---- candidate offsets per (comp, class, category) and per (comp, band) from the CTB's sums
    // (packed counts add up: at most 1,024 samples per CTB component)
    const uint32_t lam16 = kLambdaSse16[fs->qp < 0 ? 0 : (fs->qp > 51 ? 51 : fs->qp)];
    if (valid && !keep) {
        if (lane < 48) {
            const int comp = lane >> 4, q = lane & 15, cat = q & 3;
            const int v = sw[0].eo[comp][q] + sw[1].eo[comp][q] + sw[2].eo[comp][q] + sw[3].eo[comp][q];
            int o;
            S.jeo[comp][q] = sao_best_offset(sao_unpack_sum(v), sao_unpack_cnt(v), cat < 2 ? 0 : -7, cat < 2 ? 7 : 0,
                                             false, lam16, &o);
            S.oeo[comp][q] = o;
        }
        for (int t = lane; t < 96; t += 64) {
            const int comp = t >> 5, b = t & 31;
            const int v = sw[0].bo[comp][b] + sw[1].bo[comp][b] + sw[2].bo[comp][b] + sw[3].bo[comp][b];
            int o;
            S.jb[comp][b] = sao_best_offset(sao_unpack_sum(v), sao_unpack_cnt(v), -7, 7, true, lam16, &o);
            S.ob[comp][b] = o;
        }
    }
    sao_wave_sync();
    // ---- per component: best band window (lexicographic min of (cost, position) over 32 lanes)
    //      and the edge-class sums
    if (valid && !keep) {
        for (int pass = 0; pass < 2; ++pass) {
            const int comp = pass * 2 + (lane >> 5), p = lane & 31;
            const bool on = comp < 3;
            int j = 0x7fffffff;
            if (on) j = S.jb[comp][p] + S.jb[comp][(p + 1) & 31] + S.jb[comp][(p + 2) & 31] + S.jb[comp][(p + 3) & 31];
            int bp = p;
            for (int o = 16; o > 0; o >>= 1) {
                const int jo = __shfl_xor(j, o, 64), po = __shfl_xor(bp, o, 64);
                if (jo < j || (jo == j && po < bp)) {
                    j = jo;
                    bp = po;
                }
            }
            if (on && p == 0) {
                SaoCompChoice& c = S.ch[comp];
                c.j_bo = j;
                c.band = bp;
                for (int k = 0; k < 4; ++k) c.bo_off[k] = S.ob[comp][(bp + k) & 31];
            }
        }
        if (lane < 12) {
            const int comp = lane >> 2, k = lane & 3;
            SaoCompChoice& c = S.ch[comp];
            c.j_eo[k] = S.jeo[comp][4 * k] + S.jeo[comp][4 * k + 1] + S.jeo[comp][4 * k + 2] + S.jeo[comp][4 * k + 3];
            for (int q = 0; q < 4; ++q) c.eo_off[k][q] = S.oeo[comp][4 * k + q];
        }
    }
    sao_wave_sync();
    if (valid && lane == 0) {
        uint32_t w[3] = {0u, 0u, 0u};
        if (!keep) sao_combine(S.ch[0], S.ch[1], S.ch[2], lam16, w);
        S.w[0] = w[0];
        S.w[1] = w[1];
        S.w[2] = w[2];
        if (wave == 0) *reinterpret_cast<uint4*>(prm + 4 * (size_t)bid) = make_uint4(w[0], w[1], w[2], 0u);
    }
    sao_wave_sync();
    // ---- apply into the output picture; distortion over the display area
    int ey = 0, eu = 0, ev = 0;
    if (valid) {
        const uint32_t wy = S.w[0], wu = S.w[1], wv = S.w[2];
        const uint32_t sv = *(const sao_gu32*)(src_y + (size_t)(y0 + r) * g.pitch + x0 + c0);
        uint32_t packed = 0;
        const int ky = 3 * sao_eo(wy);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cat = (int)((cat_y >> (12 * j + ky)) & 7);
            const int o = sao_sample_cat(wy, (int)((cen_y >> (8 * j)) & 255), cat);
            packed |= (uint32_t)o << (8 * j);
            const int d = (int)((sv >> (8 * j)) & 255) - o;
            ey += (x0 + c0 + j < g.width && y0 + r < g.height) ? d * d : 0;
        }
        *(sao_gu32*)(fs->sao_y + (size_t)(y0 + r) * g.pitch + x0 + c0) = packed;
        const int u = sao_sample_cat(wu, (int)(cen_uv & 255), (int)((cat_u >> (3 * sao_eo(wu))) & 7));
        const int v = sao_sample_cat(wv, (int)(cen_uv >> 8), (int)((cat_v >> (3 * sao_eo(wv))) & 7));
        *(sao_gu16*)(fs->sao_uv + (size_t)yc * g.pitch + 2 * xc) = (uint16_t)(u | (v << 8));
        const uint32_t spair = *(const sao_gu16*)(src_uv + (size_t)yc * g.pitch + 2 * xc);
        const bool disp = 2 * xc < g.width && 2 * yc < g.height;
        const int du = (int)(spair & 255) - u, dv = (int)(spair >> 8) - v;
        eu = disp ? du * du : 0;
        ev = disp ? dv * dv : 0;
    }
    ey = wsum(ey);
    eu = wsum(eu);
    ev = wsum(ev);
    if (lane == 0) {
        // 4th channel: luma of units outside the quality-report mask
        const int cx = ux, cy = uy;
        const bool in_mask = cx >= fs->mask_c[0] && cx < fs->mask_c[2] && cy >= fs->mask_c[1] && cy < fs->mask_c[3];
        part[0][wave] = (unsigned long long)ey;
        part[1][wave] = (unsigned long long)eu;
        part[2][wave] = (unsigned long long)ev;
        part[3][wave] = valid && !in_mask ? (unsigned long long)ey : 0ull;
    }
    __syncthreads();
    if (threadIdx.x < 4) {  // one atomic per workgroup and channel into one of kSseSlots 64-byte slots
        // (8,100 workgroups adding into the same 4 words serialised in one L2 channel: ~100 us of
        // k_hevc_sao at 4K); k_hevc_pack sums the slots
        const int c = threadIdx.x;
        atomicAdd(fs->sse_tot + (size_t)(blockIdx.x % kSseSlots) * kSseSlotWords + c,
                  part[c][0] + part[c][1] + part[c][2] + part[c][3]);
    }
}

// Distortion of the final (deblocked) picture over the display area: one workgroup per CTU
// row, partial sums per row for k_hevc_pack.
__global__ __launch_bounds__(256) void k_hevc_sse(Geometry g, const HevcFrameState* __restrict__ fs,
                                                   const uint8_t* __restrict__ src_y, const uint8_t* __restrict__ src_uv) {
    __shared__ unsigned long long red[3][4];
    const int r = blockIdx.x, tid = threadIdx.x;
    unsigned long long e[3] = {0, 0, 0};
    const int quads = (g.width + 3) >> 2;  // dword columns (pitch is 256-aligned)
    auto acc = [&](const uint8_t* a, const uint8_t* b, int row, int q, bool chroma) {
        const uint32_t va = *reinterpret_cast<const uint32_t*>(a + (size_t)row * g.pitch + 4 * q);
        const uint32_t vb = *reinterpret_cast<const uint32_t*>(b + (size_t)row * g.pitch + 4 * q);
        for (int j = 0; j < 4; ++j) {
            if (4 * q + j >= g.width) break;
            const int d = (int)((va >> (8 * j)) & 255) - (int)((vb >> (8 * j)) & 255);
            if (!chroma)
                e[0] += (unsigned)(d * d);
            else if (j & 1)
                e[2] += (unsigned)(d * d);
            else
                e[1] += (unsigned)(d * d);
        }
    };
    const int rows = min(16, g.height - r * 16), crows = min(8, g.height / 2 - r * 8);
    const uint8_t* fy = fs->rec_y;  // the final (deblocked) picture
    const uint8_t* fuv = fs->rec_uv;
    for (int k = tid; k < rows * quads; k += 256) acc(src_y, fy, r * 16 + k / quads, k % quads, false);
    for (int k = tid; k < crows * quads; k += 256) acc(src_uv, fuv, r * 8 + k / quads, k % quads, true);
    for (int o = 32; o > 0; o >>= 1) {
        e[0] += __shfl_xor(e[0], o, 64);
        e[1] += __shfl_xor(e[1], o, 64);
        e[2] += __shfl_xor(e[2], o, 64);
    }
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = e[0];
        red[1][tid >> 6] = e[1];
        red[2][tid >> 6] = e[2];
    }
    __syncthreads();
    if (tid < 3) {
        const unsigned long long v = tid == 0 ? red[0][0] + red[0][1] + red[0][2] + red[0][3]
                                     : tid == 1 ? red[1][0] + red[1][1] + red[1][2] + red[1][3]
                                                : red[2][0] + red[2][1] + red[2][2] + red[2][3];
        fs->sse_part[tid * h264::kSsePartStride + r] = v;
    }
}

// ------------------------------------------------------------------ pack
// One workgroup per substream (a slice, or with WPP a CTU row): its payload to a 16-byte aligned
// place in the host buffer, and its (offset, length, first CTU | kSubSliceStart when it begins a
// slice) record; workgroup 0 also writes the header.
__device__ void pack_body(Geometry g, const HevcFrameState* __restrict__ fs, const uint32_t* __restrict__ nslices,
                          const int* __restrict__ slice_first, const int* __restrict__ slice_of_cu,
                          const uint8_t* __restrict__ slice_data, uint32_t slice_cap,
                          const uint32_t* __restrict__ slice_len, uint8_t* __restrict__ host_out, size_t out_bytes);

__global__ __launch_bounds__(256) void k_hevc_pack(Geometry g, const HevcFrameState* __restrict__ fs,
                                                    const uint32_t* __restrict__ nslices,
                                                    const int* __restrict__ slice_first,
                                                    const int* __restrict__ slice_of_cu,
                                                    const uint8_t* __restrict__ slice_data,
                                                    uint32_t slice_cap, const uint32_t* __restrict__ slice_len,
                                                    uint8_t* __restrict__ host_out, size_t out_bytes,
                                                    uint32_t* __restrict__ done) {
    const int tid = threadIdx.x;
    pack_body(g, fs, nslices, slice_first, slice_of_cu, slice_data, slice_cap, slice_len, host_out, out_bytes);
    // the last workgroup to finish stamps the frame's end clock into the host header (read after
    // the frame's completion event) and re-arms the counter for the next frame
    __syncthreads();
    if (tid == 0) {
        // relaxed: only the count matters (the host reads the header after the frame's completion
        // event); acq_rel put an L2 write-back (buffer_wbl2) + invalidate around it in every one of
        // the workgroups
        const uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            reinterpret_cast<HevcOutHeader*>(host_out)->t_end = wall_clock64();
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ void pack_body(Geometry g, const HevcFrameState* __restrict__ fs, const uint32_t* __restrict__ nslices,
                          const int* __restrict__ slice_first, const int* __restrict__ slice_of_cu,
                          const uint8_t* __restrict__ slice_data, uint32_t slice_cap,
                          const uint32_t* __restrict__ slice_len, uint8_t* __restrict__ host_out, size_t out_bytes) {
    __shared__ uint32_t red[256];
    __shared__ unsigned long long red64[4][256];
    const int s = blockIdx.x, tid = threadIdx.x;
    const bool wpp = fs->wpp != 0;
    const int cw = ctb_cols(g.mb_w);
    const int num_slices = wpp ? ctb_rows(g.mb_h) : (int)*nslices;  // substreams
    if (s >= num_slices) return;
    // offset of this slice: sum of the 16-byte rounded lengths before it
    uint32_t part = 0;
    for (int k = tid; k < s; k += 256) part += (min(slice_len[k], slice_cap) + 15) & ~15u;
    red[tid] = part;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    const uint32_t off = red[0];
    const uint32_t len = slice_len[s];
    const bool fits = len <= slice_cap && (size_t)off + ((len + 15) & ~15u) <= out_bytes;
    if (fits) {
        const uint4* src = reinterpret_cast<const uint4*>(slice_data + (size_t)s * slice_cap);
        uint4* dst = reinterpret_cast<uint4*>(host_out + kOutPayloadOffset + off);
        for (uint32_t k = tid; k < (len + 15) / 16; k += 256) dst[k] = src[k];
    }
    if (tid == 0) {
        uint32_t* offs = reinterpret_cast<uint32_t*>(host_out + sizeof(HevcOutHeader));
        offs[s] = off;
        offs[kMaxSlices + s] = len;
        const int fc = wpp ? s * cw : slice_first[s];  // first CTB
        const bool starts = !wpp || slice_first[slice_of_cu[fc]] == fc;
        offs[2 * kMaxSlices + s] = (uint32_t)fc | (starts ? kSubSliceStart : 0u);
    }
    if (s != 0) return;
    // header: totals, overflow, distortion
    uint32_t tot = 0, ovf = 0;
    for (int k = tid; k < num_slices; k += 256) {
        tot += (min(slice_len[k], slice_cap) + 15) & ~15u;
        ovf |= slice_len[k] > slice_cap ? 1u : 0u;
    }
    // distortion partials: 4 channels (the 4th, masked luma, only from k_hevc_sao), loads batched
    unsigned long long e[4] = {0, 0, 0, 0};
    if (fs->sao) {  // totals accumulated by k_hevc_sao (a serial walk over 8,100 partials x 4 was
                    // ~30 us at the end of the entropy stream)
        if (tid < 4 * kSseSlots) e[tid & 3] = fs->sse_tot[(size_t)(tid >> 2) * kSseSlotWords + (tid & 3)];
    } else {
        const int num_sse_parts = fs->n_sse_parts;
#pragma unroll 4
        for (int k = tid; k < num_sse_parts; k += 256)
            for (int c = 0; c < 3; ++c) e[c] += fs->sse_part[c * h264::kSsePartStride + k];
    }
    // wave reductions (the former thread-0 loop over 256 x 5 LDS values was ~20 us of the
    // entropy stream's tail), then 4 partials per value
    const int lane = tid & 63, wv = tid >> 6;
    for (int o = 32; o > 0; o >>= 1) {
        tot += __shfl_xor(tot, o, 64);
        ovf |= __shfl_xor(ovf, o, 64);
        for (int c = 0; c < 4; ++c) e[c] += __shfl_xor(e[c], o, 64);
    }
    __syncthreads();
    if (lane == 0) {
        red[wv] = tot | (ovf << 31);
        for (int c = 0; c < 4; ++c) red64[c][wv] = e[c];
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t T = 0, O = 0;
        unsigned long long E[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k) {
            T += red[k] & 0x7fffffffu;
            O |= red[k] >> 31;
            for (int c = 0; c < 4; ++c) E[c] += red64[c][k];
        }
        HevcOutHeader& h = *reinterpret_cast<HevcOutHeader*>(host_out);  // not t_start / t_end
        h.total_bytes = T;
        h.num_slices = (uint32_t)num_slices;
        h.overflow = (O || T > out_bytes) ? 1u : 0u;
        h.deblocked = (uint32_t)fs->deblock_on;
        for (int c = 0; c < 3; ++c) h.sse[c] = E[c];
        h.sse_masked = E[3];
    }
}

__global__ __launch_bounds__(64) void k_hevc_publish(HevcFrameState* __restrict__ dfs, HevcFrameState v,
                                                      h264::FrameState* __restrict__ dme, h264::FrameState vme,
                                                      int has_me, uint64_t* __restrict__ t_start) {
    const int t = threadIdx.x;
    if (t == 0 && t_start) *t_start = wall_clock64();
    const uint32_t* a = reinterpret_cast<const uint32_t*>(&v);
    for (int i = t; i < (int)(sizeof(HevcFrameState) / 4); i += 64) reinterpret_cast<uint32_t*>(dfs)[i] = a[i];
    if (has_me) {
        const uint32_t* m = reinterpret_cast<const uint32_t*>(&vme);
        for (int i = t; i < (int)(sizeof(h264::FrameState) / 4); i += 64) reinterpret_cast<uint32_t*>(dme)[i] = m[i];
    }
}

// IDR pictures with temporal AQ: copy the source luma to save_src.  The destination is read from
// the device copy of the frame state, so a captured graph stays valid while the two source
// buffers alternate (a memcpy node would freeze the pointer of the frame it was captured for).
__global__ __launch_bounds__(256) void k_hevc_save_src(Geometry g, const HevcFrameState* __restrict__ fs,
                                                        const uint8_t* __restrict__ src_y) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // 16-byte chunk
    const size_t n = (size_t)g.pitch * g.coded_h / 16;
    if (i < n) reinterpret_cast<uint4*>(fs->save_src)[i] = reinterpret_cast<const uint4*>(src_y)[i];
}

}  // namespace

void launch_hevc_save_src(const Geometry& g, const HevcDeviceBuffers& b, const uint8_t* src_y, hipStream_t s) {
    const size_t n = (size_t)g.pitch * g.coded_h / 16;  // pitch is a multiple of 256
    hipLaunchKernelGGL(k_hevc_save_src, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, b.fs, src_y);
}

void launch_hevc_inter(const Geometry& g, const HevcDeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                       hipStream_t s) {
    const int nctb = ctb_cols(g.mb_w) * ctb_rows(g.mb_h);
    hipLaunchKernelGGL(k_hevc_inter, dim3(nctb), dim3(256), 0, s, g, b.fs, b.me.mb, src_y, src_uv, b.cu, b.coef, b.cost,
                       b.qpc);
}

void launch_hevc_intra(const Geometry& g, const HevcDeviceBuffers& b, int slice_rows, int num_slices,
                       const uint8_t* src_y, const uint8_t* src_uv, hipStream_t s) {
    const int nctb = ctb_cols(g.mb_w) * ctb_rows(g.mb_h);
    hipLaunchKernelGGL(k_hevc_intra_modes, dim3(nctb), dim3(256), 0, s, g, b.fs, src_y, b.imode);
    const size_t lds = (size_t)slice_rows * 2 * g.coded_w;
    hipLaunchKernelGGL(k_hevc_intra, dim3(num_slices), dim3(64 * slice_rows), lds, s, g, b.fs, src_y, src_uv, b.cu,
                       b.coef, b.imode, b.qpc);
}

void launch_hevc_layout(const Geometry& g, const HevcDeviceBuffers& b, bool idr, int max_slices, int slice_cost, bool deblock,
                        bool sao, const uint8_t* src_y, const uint8_t* src_uv, hipStream_t s, bool deblock_auto) {
    const int ncu = g.mb_w * g.mb_h;
    const int cw = ctb_cols(g.mb_w), nctb = cw * ctb_rows(g.mb_h);
    hipLaunchKernelGGL(k_hevc_layout, dim3((nctb + kScanTile - 1) / kScanTile), dim3(1024), 0, s, b.fs, b.cost, nctb, cw,
                       max_slices, slice_cost, b.slice_first, b.slice_of_cu, b.nslices);
    if (!idr)
        hipLaunchKernelGGL(k_hevc_decide, dim3((nctb + 255) / 256), dim3(256), 0, s, g, b.me.mb, b.slice_first,
                           b.slice_of_cu, b.cu);
    // QpY chain: the deblocking filter's QP and the entropy coder's QP predictor
    hipLaunchKernelGGL(k_hevc_qpy, dim3(std::max(max_slices, ctb_rows(g.mb_h))), dim3(256), 0, s, g, b.fs, b.cu, b.qpc,
                       b.slice_first, b.nslices, b.qp_pred, b.qpy);
    if (deblock) {
        if (deblock_auto)
            hipLaunchKernelGGL(k_hevc_db_auto, dim3((ncu + 1023) / 1024), dim3(1024), 0, s, g, b.fs, b.me.mb, b.db_state);
        for (int dir = 0; dir < 2; ++dir)
            hipLaunchKernelGGL(k_hevc_deblock, dim3((ncu * 4 + 255) / 256), dim3(256), 0, s, g, b.fs, b.cu, b.qpy, dir);
    }
    if (sao)  // SAO per CTB, with the final distortion (one partial per CTB)
        hipLaunchKernelGGL(k_hevc_sao, dim3(nctb), dim3(256), 0, s, g, b.fs, src_y, src_uv, b.cu, b.sao);
    else if (deblock)
        hipLaunchKernelGGL(k_hevc_sse, dim3(g.mb_h), dim3(256), 0, s, g, b.fs, src_y, src_uv);
}

void launch_hevc_entropy(const Geometry& g, const HevcDeviceBuffers& b, int max_slices, uint8_t* host_out,
                         hipStream_t s) {
    const int npos = 4 * ctb_cols(g.mb_w) * ctb_rows(g.mb_h);  // coding positions
    if ((npos + kScanTile - 1) / kScanTile > kMaxScanTiles) throw std::invalid_argument("hevc: picture too large");
    hipLaunchKernelGGL(k_hevc_bins, dim3(npos), dim3(64), 0, s, g, b.fs, b.cu, b.coef, b.sao, b.slice_first,
                       b.slice_of_cu, b.nslices, b.qp_pred, b.tok, b.ntok);
    hipLaunchKernelGGL(k_hevc_tokscan, dim3((npos + kScanTile - 1) / kScanTile), dim3(1024), 0, s, b.ntok, npos,
                       b.tok_off);
    hipLaunchKernelGGL(k_hevc_tokgather, dim3((npos + 3) / 4), dim3(256), 0, s, b.tok, b.ntok, b.tok_off, npos,
                       b.tok_dense);
    const int max_subs = std::max(max_slices, ctb_rows(g.mb_h));  // substreams: slices, or CTB rows with WPP
    hipLaunchKernelGGL(k_hevc_arith, dim3(max_subs), dim3(64), 0, s, g, b.fs, b.tok_dense, b.tok_off,
                       b.slice_first, b.slice_of_cu, b.nslices, b.slice_data, b.slice_cap, b.slice_len, b.slice_clk);
    hipLaunchKernelGGL(k_hevc_pack, dim3(max_subs), dim3(256), 0, s, g, b.fs, b.nslices, b.slice_first, b.slice_of_cu,
                       b.slice_data, b.slice_cap, b.slice_len, host_out, b.out_bytes, b.pack_done);
}

void launch_hevc_publish(const HevcDeviceBuffers& b, const HevcFrameState& fs, const h264::FrameState* me_fs,
                         uint64_t* t_start, hipStream_t s) {
    static_assert(sizeof(HevcFrameState) % 4 == 0 && sizeof(h264::FrameState) % 4 == 0, "word copies");
    const h264::FrameState none{};
    hipLaunchKernelGGL(k_hevc_publish, dim3(1), dim3(64), 0, s, b.fs, fs, b.me.fs, me_fs ? *me_fs : none,
                       me_fs ? 1 : 0, t_start);
}

}  // namespace hevc
}  // namespace mx
