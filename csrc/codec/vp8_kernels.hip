// HIP analysis kernels of the VP8 encoder (RFC 6386; WEBRTC_ENCODER=vp8enc, reference
// README.md:21,35): every decision and sample of CpuVp8Encoder::analyse (vp8_cpu.cpp), on the GPU.
//
//   P frame:   k_vp8_pad (or the H.264 k_hpel planes with subpel) -> k_me_full (shared with
//              H.264) -> k_vp8_inter [-> k_vp8_lf] -> k_vp8_gather
//   key frame: k_vp8_key [-> k_vp8_lf] -> k_vp8_gather
//   (k_vp8_lf: the loop filter, when the frame's levels are not all zero)
//
// One 64-lane wave codes one macroblock: lanes 0..15 own the luma 4x4 blocks, 16..23 the chroma
// blocks, lane 24 the second-order Y2 block -- the block index of a lane is its token block index,
// so the non-zero mask is one ballot.  The dead-zone division of the quantiser is an exact
// multiply-high (Vp8FrameState::qm, exact for every coefficient the transforms produce).
// Key frames predict from reconstructed neighbours: one wave per macroblock row walks its row,
// the row below follows one macroblock behind, fed the bottom sample rows through a hand-off
// line of epoch-tagged 64-bit agent-scope atomics (bounded polls; a timeout raises the mapped
// error word instead of hanging; no release fence per macroblock).  (Rows stepping in lockstep groups with LDS hand-off lines
// measured slower -- 2.0 ms with 4-row, 4.1 ms with 16-row groups against 1.41 ms at 1080p:
// the per-macroblock chain, not the hand-off, bounds the key frame; profiles/r04_vp8/NOTES.md.)
// Inter frames segment their macroblocks by the temporal AQ classes (vp8_core.h Seg).  The boolean coder runs on host threads (vp8_bitstream.cpp);
// k_vp8_gather hands it only the coded macroblocks' levels, compacted per row, in mapped memory.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../common/hip_check.h"
#include "h264_core.h"
#include "h264_gpu.h"
#include "h264_mb.h"
#include "vp8_encoder.h"

namespace mx {
namespace vp8 {

namespace {

typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr unsigned kSpinLimit = 1u << 22;

// Wave sum, every lane gets it (whole wave active): DPP within rows of 16 (quad_perm
// [1,0,3,2], [2,3,0,1], row_ror 4, row_ror 8), then v_permlane16/32_swap with both operands = v,
// whose pair holds {v, v ^ 16} / {v, v ^ 32} -- no ds_bpermute round trips.
__device__ __forceinline__ int wsum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
    const auto r16 = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    const uint32_t u = r16[0] + r16[1];
    const auto r32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return (int)(r32[0] + r32[1]);
}

// dead-zone quantiser of vp8_core.h quantize(): (3|c| + q) / (3q) as a multiply-high
__device__ __forceinline__ int qz(int c, int q, uint32_t m) {
    const int a = c < 0 ? -c : c;
    int l = (int)__umulhi((uint32_t)(3 * a + q), m);
    l = l > 2048 ? 2048 : l;
    return c < 0 ? -l : l;
}

// Staged samples of the macroblock being coded (one wave).
struct MbLds {
    uint8_t src[256], pred[256], rec[256];
    uint8_t su[64], sv[64], pu[64], pv[64], ru[64], rv[64];
    int dc[16], dcr[16];
};

// Transform, quantise and reconstruct the staged macroblock (s.src / s.pred -> s.rec, levels to
// lv[400]); returns the non-zero block mask (bit b = block b), wave-uniform.  code_luma16 +
// code_chroma8 of vp8_core.h, one block per lane.
// drop_lambda >= 0 (inter macroblocks): vp8_drop_residual may turn the macroblock into prediction
// only (levels zero, reconstruction = prediction) -- the decision is wave-uniform.
// luma_coded (B_PRED key-frame macroblocks): the luma is coded already (levels, s.rec) -- only the
// chroma blocks here, and a zero Y2 block.
__device__ uint32_t code_mb(MbLds& s, const Vp8FrameState& F, int16_t* __restrict__ lv, int lane,
                            int drop_lambda = -1, int seg = 0, bool luma_coded = false) {
    const int32_t* Fq = F.q[seg];      // the macroblock's segment quantiser (wave-uniform)
    const uint32_t* Fqm = F.qm[seg];
    int lvl[16], dq[16];
    bool nz = false;
    int st_lsad = 0, st_dp = 0, st_dc = 0, st_bits = 0;  // drop statistics (luma lanes, Y2 lane)
    const bool luma = lane < 16 && !luma_coded, chroma = lane >= 16 && lane < 24;
#pragma unroll
    for (int k = 0; k < 16; ++k) lvl[k] = dq[k] = 0;
    if (luma || chroma) {
        int in[16];
        if (luma) {
            const int bx = lane & 3, by = lane >> 2;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 16 + bx * 4 + j;
                    in[i * 4 + j] = (int)s.src[o] - (int)s.pred[o];
                }
        } else {
            const int b = (lane - 16) & 3, bx = b & 1, by = b >> 1;
            const uint8_t* S = lane < 20 ? s.su : s.sv;
            const uint8_t* P = lane < 20 ? s.pu : s.pv;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 8 + bx * 4 + j;
                    in[i * 4 + j] = (int)S[o] - (int)P[o];
                }
        }
        if (luma)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                st_lsad += in[k] < 0 ? -in[k] : in[k];
                st_dp += in[k] * in[k];
            }
        int coef[16];
        fdct4x4(in, coef);
        if (luma) s.dc[lane] = coef[0];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (luma && k == 0) continue;  // the DC travels in Y2
            const int pos = kZigzag[k];
            const int qi = luma ? 1 : (k == 0 ? 4 : 5);
            const int q = Fq[qi];
            const int l = qz(coef[pos], q, Fqm[qi]);
            lvl[k] = l;
            dq[pos] = l * q;
            nz |= l != 0;
        }
    }
    __syncthreads();
    if (lane == kY2 && !luma_coded) {
        int dcv[16], y2[16], y2q[16], dcr[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) dcv[b] = s.dc[b];
        fwht4x4(dcv, y2);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int pos = kZigzag[k];
            const int qi = k == 0 ? 2 : 3;
            const int l = qz(y2[pos], Fq[qi], Fqm[qi]);
            lvl[k] = l;
            y2q[pos] = l * Fq[qi];
            nz |= l != 0;
        }
        iwht4x4(y2q, dcr);
#pragma unroll
        for (int b = 0; b < 16; ++b) s.dcr[b] = dcr[b];
        int n = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) n += lvl[k] != 0;
        st_bits = (int)vp8_block_bits(n);
    }
    __syncthreads();
    if (luma || chroma) {
        if (luma) dq[0] = s.dcr[lane];
        int r[16];
        idct4x4(dq, r);
        if (luma) {
            const int bx = lane & 3, by = lane >> 2;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 16 + bx * 4 + j;
                    const int v = v8_clamp255((int)s.pred[o] + r[i * 4 + j]);
                    s.rec[o] = (uint8_t)v;
                    const int e = (int)s.src[o] - v;
                    st_dc += e * e;
                }
            int n = 0;
#pragma unroll
            for (int k = 1; k < 16; ++k) n += lvl[k] != 0;
            st_bits = (int)vp8_block_bits(n);
        } else {
            const int b = (lane - 16) & 3, bx = b & 1, by = b >> 1;
            const uint8_t* P = lane < 20 ? s.pu : s.pv;
            uint8_t* R = lane < 20 ? s.ru : s.rv;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 8 + bx * 4 + j;
                    R[o] = (uint8_t)v8_clamp255((int)P[o] + r[i * 4 + j]);
                }
        }
    }
    bool drop = false;
    if (drop_lambda >= 0) {  // wave-uniform
        const uint32_t lsad = (uint32_t)wsum(st_lsad), bits = (uint32_t)wsum(st_bits);
        drop = vp8_drop_residual(lsad, (long long)wsum(st_dp), (long long)wsum(st_dc), bits, drop_lambda);
    }
    if (drop) {
        nz = false;
#pragma unroll
        for (int k = 0; k < 16; ++k) lvl[k] = 0;
        if (luma) {
            const int bx = lane & 3, by = lane >> 2;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 16 + bx * 4 + j;
                    s.rec[o] = s.pred[o];
                }
        } else if (chroma) {
            const int b = (lane - 16) & 3, bx = b & 1, by = b >> 1;
            const uint8_t* P = lane < 20 ? s.pu : s.pv;
            uint8_t* R = lane < 20 ? s.ru : s.rv;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int o = (by * 4 + i) * 8 + bx * 4 + j;
                    R[o] = P[o];
                }
        }
    }
    if (lane < kBlocks && (luma || lane >= 16)) {
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = (uint32_t)(uint16_t)lvl[2 * k] | ((uint32_t)(uint16_t)lvl[2 * k + 1] << 16);
        uint4* d = reinterpret_cast<uint4*>(lv + lane * 16);
        d[0] = make_uint4(w[0], w[1], w[2], w[3]);
        d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
    const uint32_t mask = (uint32_t)__ballot(nz) & ((1u << kBlocks) - 1);
    __syncthreads();
    return mask;
}

// Source of the macroblock at (x0, y0) into LDS: luma one dword per lane, chroma (interleaved
// rows) deinterleaved by the first 32 lanes.
__device__ __forceinline__ void stage_src(MbLds& s, const h264::Geometry& g, const uint8_t* __restrict__ sy,
                                          const uint8_t* __restrict__ suv, int x0, int y0, int lane) {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    *reinterpret_cast<uint32_t*>(s.src + r * 16 + c4) =
        *reinterpret_cast<const uint32_t*>(sy + (size_t)(y0 + r) * g.pitch + x0 + c4);
    if (lane < 32) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(suv + (size_t)(y0 / 2 + r) * g.pitch + x0 + c4);
        const int o = r * 8 + (c4 >> 1);
        s.su[o] = (uint8_t)w;  // U V U V
        s.sv[o] = (uint8_t)(w >> 8);
        s.su[o + 1] = (uint8_t)(w >> 16);
        s.sv[o + 1] = (uint8_t)(w >> 24);
    }
}

// Reconstruction of the staged macroblock to the picture, and its distortion over the display
// area (Y, U, V) -- wave-uniform sums.
__device__ __forceinline__ void store_rec(const MbLds& s, const h264::Geometry& g, const Vp8FrameState& F, int x0,
                                          int y0, int lane, uint32_t sse[3]) {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    *reinterpret_cast<uint32_t*>(F.rec_y + (size_t)(y0 + r) * g.pitch + x0 + c4) =
        *reinterpret_cast<const uint32_t*>(s.rec + r * 16 + c4);
    int ey = 0;
    if (y0 + r < g.height)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = (int)s.src[r * 16 + c4 + j] - (int)s.rec[r * 16 + c4 + j];
            ey += x0 + c4 + j < g.width ? e * e : 0;
        }
    if (lane < 32) {
        const int o = r * 8 + (c4 >> 1);
        const uint32_t w = (uint32_t)s.ru[o] | ((uint32_t)s.rv[o] << 8) | ((uint32_t)s.ru[o + 1] << 16) |
                           ((uint32_t)s.rv[o + 1] << 24);
        *reinterpret_cast<uint32_t*>(F.rec_uv + (size_t)(y0 / 2 + r) * g.pitch + x0 + c4) = w;
    }
    const int cx = lane & 7, cy = lane >> 3;
    const bool vis = 2 * (x0 / 2 + cx) < g.width && 2 * (y0 / 2 + cy) < g.height;
    const int eu = (int)s.su[cy * 8 + cx] - (int)s.ru[cy * 8 + cx];
    const int ev = (int)s.sv[cy * 8 + cx] - (int)s.rv[cy * 8 + cx];
    sse[0] = (uint32_t)wsum(ey);
    sse[1] = (uint32_t)wsum(vis ? eu * eu : 0);
    sse[2] = (uint32_t)wsum(vis ? ev * ev : 0);
}

// store_rec without the stores: the reconstruction's words (luma one per lane, chroma one per lane
// < 32) and the distortion, for a store issued later (k_vp8_key defers it past the next poll)
__device__ __forceinline__ void rec_words(const MbLds& s, const h264::Geometry& g, int x0, int y0, int lane,
                                          uint32_t& wy, uint32_t& wuv, uint32_t sse[3]) {
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    wy = *reinterpret_cast<const uint32_t*>(s.rec + r * 16 + c4);
    int ey = 0;
    if (y0 + r < g.height)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = (int)s.src[r * 16 + c4 + j] - (int)s.rec[r * 16 + c4 + j];
            ey += x0 + c4 + j < g.width ? e * e : 0;
        }
    const int o = (r & 7) * 8 + (c4 >> 1);
    wuv = (uint32_t)s.ru[o] | ((uint32_t)s.rv[o] << 8) | ((uint32_t)s.ru[o + 1] << 16) | ((uint32_t)s.rv[o + 1] << 24);
    const int cx = lane & 7, cy = lane >> 3;
    const bool vis = 2 * (x0 / 2 + cx) < g.width && 2 * (y0 / 2 + cy) < g.height;
    const int eu = (int)s.su[cy * 8 + cx] - (int)s.ru[cy * 8 + cx];
    const int ev = (int)s.sv[cy * 8 + cx] - (int)s.rv[cy * 8 + cx];
    sse[0] = (uint32_t)wsum(ey);
    sse[1] = (uint32_t)wsum(vis ? eu * eu : 0);
    sse[2] = (uint32_t)wsum(vis ? ev * ev : 0);
}

__device__ __forceinline__ void store_record(Vp8Mb* __restrict__ rec, int mvx, int mvy, int ymode, int uvmode,
                                             uint32_t nz, const uint32_t sse[3], int lane, int seg = 0,
                                             uint32_t bmodes_hi = 0) {
    if (lane == 0) {
        Vp8Mb m;
        m.mvx = (int16_t)mvx;
        m.mvy = (int16_t)mvy;
        m.ymode = (uint8_t)ymode;
        m.uvmode = (uint8_t)uvmode;
        m.seg = (uint8_t)seg;
        m.pad1 = 0;
        m.nz = nz;
        m.slot = 0;
        m.sse[0] = sse[0];
        m.sse[1] = sse[1];
        m.sse[2] = sse[2];
        m.bmodes_hi = bmodes_hi;
        *rec = m;
    }
}

// ------------------------------------------------------------------ P frames
// Padded full-sample reference (edge replicated, kHpelPad around the coded picture) for k_me_full
// and the luma prediction; one dword per thread.
__global__ __launch_bounds__(256) void k_vp8_pad(h264::Geometry g, const Vp8States* __restrict__ st) {
    const Vp8FrameState& F = st->v;
    const int W = g.coded_w + 2 * h264::kHpelPad, H = g.coded_h + 2 * h264::kHpelPad;
    const int x4 = (blockIdx.x * 256 + threadIdx.x) * 4, y = blockIdx.y;
    if (x4 >= W || y >= H) return;
    const int sy = min(max(y - h264::kHpelPad, 0), g.coded_h - 1);
    const uint8_t* row = F.ref_y + (size_t)sy * g.pitch;
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int sx = min(max(x4 + k - h264::kHpelPad, 0), g.coded_w - 1);
        w |= (uint32_t)row[sx] << (8 * k);
    }
    uint8_t* dst = F.hp_f - (size_t)h264::kHpelPad * F.hp_pitch - h264::kHpelPad;
    *reinterpret_cast<uint32_t*>(dst + (size_t)y * F.hp_pitch + x4) = w;
}

// Chroma inter prediction sample: sixtap_px of vp8_core.h with the pass of a zero phase skipped
// (the 128 tap is exact), so the common full-sample cases load 1 or 6 samples instead of 36.
template <class A>
__device__ __forceinline__ int chroma_px(const A& at, int x, int y, int fx, int fy) {
    if ((fx | fy) == 0) return at(x, y);
    if (fy == 0) {
        int h = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) h += kSubpel[fx][k] * at(x - 2 + k, y);
        return v8_clamp255((h + 64) >> 7);
    }
    if (fx == 0) {
        int v = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) v += kSubpel[fy][r] * at(x, y - 2 + r);
        return v8_clamp255((v + 64) >> 7);
    }
    return sixtap_px(at, x, y, fx, fy);
}

__global__ __launch_bounds__(64) void k_vp8_inter(h264::Geometry g, const Vp8States* __restrict__ st,
                                                   const uint8_t* __restrict__ src_y,
                                                   const uint8_t* __restrict__ src_uv,
                                                   const h264::MbInfo* __restrict__ me, Vp8Mb* __restrict__ mbs,
                                                   int16_t* __restrict__ lv, int* __restrict__ ilist) {
    __shared__ MbLds s;
    const Vp8FrameState& F = st->v;
    const int mbi = blockIdx.x, lane = threadIdx.x;
    if (mbi == 0 && lane == 0) ilist[0] = 0;  // the intra pass's candidate count (k_vp8_intra_cand)
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w, x0 = mbx * 16, y0 = mby * 16;
    int lo_x, hi_x, lo_y, hi_y;
    mv_bounds(g.mb_w, g.mb_h, mbx, mby, &lo_x, &hi_x, &lo_y, &hi_y);
    // the search's quarter-sample vector (full samples without subpel) in VP8's 1/8-sample units,
    // kept inside the range the decoder never clamps (inter_vector, as the CPU encoder)
    int mvx, mvy;
    inter_vector(me[mbi].mvx, me[mbi].mvy, lo_x, hi_x, lo_y, hi_y, &mvx, &mvy);
    mvx = __builtin_amdgcn_readfirstlane(mvx);
    mvy = __builtin_amdgcn_readfirstlane(mvy);
    const int ix = mvx >> 3, iy = mvy >> 3;
    stage_src(s, g, src_y, src_uv, x0, y0, lane);
    {  // luma prediction: the padded reference covers every legal vector (mv_bounds) and its taps
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        const uint8_t* base = F.hp_f;
        const int pitch = F.hp_pitch;
        if (((mvx | mvy) & 7) == 0) {
            const uint8_t* p = base + (ptrdiff_t)(y0 + r + iy) * pitch + x0 + c4 + ix;
#pragma unroll
            for (int j = 0; j < 4; ++j) s.pred[r * 16 + c4 + j] = p[j];
        } else {  // six-tap (18.3), the 2-D filter of sixtap_px with a zero phase's pass skipped
            auto at = [&](int xx, int yy) { return (int)base[(ptrdiff_t)yy * pitch + xx]; };
#pragma unroll
            for (int j = 0; j < 4; ++j)
                s.pred[r * 16 + c4 + j] = (uint8_t)chroma_px(at, x0 + c4 + j + ix, y0 + r + iy, mvx & 7, mvy & 7);
        }
    }
    // temporal class (h264_mb.h temporal_class) -> segment: the source against the previous source
    // displaced by the vector; this macroblock's source becomes the next frame's previous source
    int seg = kSegNormal;
    if (F.segmented) {  // frame-uniform
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(s.src + r * 16 + c4);
        int tsad = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            tsad += abs((int)((sw >> (8 * j)) & 0xff) -
                        h264::ref_px(F.prev_src, g.pitch, g.coded_w, g.coded_h, x0 + c4 + j + ix, y0 + r + iy));
        *reinterpret_cast<uint32_t*>(F.save_src + (size_t)(y0 + r) * g.pitch + x0 + c4) = sw;
        seg = seg_of_tclass(h264::temporal_class((uint32_t)wsum(tsad), mvx == 0 && mvy == 0));  // wave-uniform
    }
    const int cvx = chroma_mv(mvx), cvy = chroma_mv(mvy);
    {
        const int cx = lane & 7, cy = lane >> 3, cw = g.coded_w / 2, ch = g.coded_h / 2;
        const uint8_t* ref = F.ref_uv;
        const int pitch = g.pitch;
        auto at_u = [&](int xx, int yy) {
            xx = min(max(xx, 0), cw - 1);
            yy = min(max(yy, 0), ch - 1);
            return (int)ref[(size_t)yy * pitch + 2 * xx];
        };
        auto at_v = [&](int xx, int yy) {
            xx = min(max(xx, 0), cw - 1);
            yy = min(max(yy, 0), ch - 1);
            return (int)ref[(size_t)yy * pitch + 2 * xx + 1];
        };
        const int px = x0 / 2 + cx + (cvx >> 3), py = y0 / 2 + cy + (cvy >> 3);
        s.pu[cy * 8 + cx] = (uint8_t)chroma_px(at_u, px, py, cvx & 7, cvy & 7);
        s.pv[cy * 8 + cx] = (uint8_t)chroma_px(at_v, px, py, cvx & 7, cvy & 7);
    }
    __syncthreads();
    int psad = 0;  // the luma prediction SAD: the intra pass compares against it
    {
        const int r = lane >> 2, c4 = (lane & 3) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) psad += abs((int)s.src[r * 16 + c4 + j] - (int)s.pred[r * 16 + c4 + j]);
    }
    psad = wsum(psad);
    const uint32_t nz = code_mb(s, F, lv + (size_t)mbi * kCoefPerMb, lane, F.drop_lambda, seg);
    uint32_t sse[3];
    store_rec(s, g, F, x0, y0, lane, sse);
    store_record(mbs + mbi, mvx, mvy, kInter, kDcPred, nz, sse, lane, seg, (uint32_t)psad);
}


// Key frames with temporal classes: the source luma into the frame state's save buffer (the
// pointer read on the device, as h264 k_save_src), one dword per thread.
__global__ __launch_bounds__(256) void k_vp8_save_src(h264::Geometry g, const Vp8States* __restrict__ st,
                                                      const uint8_t* __restrict__ src_y) {
    const int x4 = (blockIdx.x * 256 + threadIdx.x) * 4, y = blockIdx.y;
    if (x4 >= g.coded_w || y >= g.coded_h) return;
    const size_t o = (size_t)y * g.pitch + x4;
    *reinterpret_cast<uint32_t*>(st->v.save_src + o) = *reinterpret_cast<const uint32_t*>(src_y + o);
}

// ------------------------------------------------------------------ key frames
struct KeyEdges {
    int ay[16], ly[16], au[8], lu[8], av[8], lvv[8];
    int cy, cu, cv;
};
__device__ __forceinline__ int pred_of(int mode, int above, int left, int corner, int dc) {
    switch (mode) {
        case kVPred:
            return above;
        case kHPred:
            return left;
        case kTmPred:
            return v8_clamp255(left + above - corner);
        default:
            return dc;
    }
}

__device__ __forceinline__ int dc_value(int sum, int cnt, int log2n) {
    if (cnt == 0) return 128;
    const int shift = log2n + cnt;
    return (sum + (1 << (shift - 1))) >> shift;
}

// B_PRED sub-block steps of k_vp8_key: the edge array (vp8_core.h bpred_edge)
struct BpLds {
    int X[16];
};
__device__ __forceinline__ void wave_lds_sync() {  // this wave's LDS writes before its later reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// raster position -> scan index (the inverse of kZigzag), 4 bits each
constexpr uint64_t kInvZigzagPacked = 0xFEA9DB83C7426510ull;
// v[i] of i in 0..3 as bitwise blends (no select the compiler could turn into a branch)
__device__ __forceinline__ int pick4(int i, int a, int b, int c, int d) {
    return (a & -(int)(i == 0)) | (b & -(int)(i == 1)) | (c & -(int)(i == 2)) | (d & -(int)(i == 3));
}
// quad broadcast of lane 4 (l / 4) + k; rotation within a row of 16: lane i <- lane (i - n) & 15
template <int k>
__device__ __forceinline__ int qbc(int v) { return __builtin_amdgcn_mov_dpp(v, k * 0x55, 0xF, 0xF, false); }
template <int n>
__device__ __forceinline__ int rror(int v) { return __builtin_amdgcn_mov_dpp(v, 0x120 + n, 0xF, 0xF, false); }
// the values of column c (rows 0..3) for lane 4 r + c of every 16-lane row: rows r, r-1, r-2, r-3
// arrive by rotations 0 / 4 / 8 / 12 and are put in row order with bitwise blends (no selects
// of DPP results: the compiler may sink those into divergent branches)
__device__ __forceinline__ void col4(int v, int r, int out[4]) {
    const int v1 = rror<4>(v), v2 = rror<8>(v), v3 = rror<12>(v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int d = (r - k) & 3;
        out[k] = (v & -(int)(d == 0)) | (v1 & -(int)(d == 1)) | (v2 & -(int)(d == 2)) | (v3 & -(int)(d == 3));
    }
}

// B_PRED luma of the staged macroblock in its planned modes (vp8_core.h bpred_code): 16 sub-blocks
// in raster order; per sub-block lanes 0..14 gather the edge array from s.rec / the edges, then
// every 16-lane row computes the sub-block (lane 4 r + c: sample (c, r)) -- prediction, forward
// DCT (rows by quad broadcasts, columns by row rotations), quantiser, inverse DCT -- and lanes
// 0..15 store the levels of block b and the reconstruction into s.rec.  No workgroup barrier:
// one wave, its LDS operations in order.  taplo / taphi: kBPredTap of this lane's sample for the
// modes B_VE .. B_HE / B_RD .. B_HU, a byte each.  Returns the blocks' non-zero bits.
__device__ uint32_t bpred_code_gpu(MbLds& s, BpLds& B, const KeyEdges& E, const Vp8FrameState& F,
                                   int16_t* __restrict__ lv, int lane, int mbx, int mby, uint32_t lo, uint32_t hi,
                                   uint32_t taplo, uint32_t taphi) {
    const bool top = mby == 0, left = mbx > 0;
    const int q = lane & 15, r = q >> 2, c = q & 3;
    const int qdc = F.q[0][0], qac = F.q[0][1];
    const uint32_t mdc = F.qm[0][0], mac = F.qm[0][1];
    const int kq = (int)((kInvZigzagPacked >> (4 * q)) & 15u);
    uint32_t nz = 0;
    for (int b = 0; b < 16; ++b) {
        const int bx = b & 3, by = b >> 2, xs = bx * 4, ys = by * 4;
        const int bm = (int)(((b < 8 ? lo >> (4 * b) : hi >> (4 * (b - 8)))) & 15u);  // (uniform)
        if (lane < 15) {  // X: L3 L3 L2 L1 L0 P A0 .. A7 A7
            int v;
            if (lane <= 4) {
                const int j = lane == 0 ? 3 : 4 - lane;
                v = bx > 0 ? s.rec[(ys + j) * 16 + xs - 1] : (left ? E.ly[ys + j] : 129);
            } else if (lane == 5) {
                v = (top && by == 0) ? 127
                    : ((!left && bx == 0) ? 129
                                          : (by > 0 ? (bx > 0 ? s.rec[(ys - 1) * 16 + xs - 1] : E.ly[ys - 1])
                                                    : (bx > 0 ? E.ay[xs - 1] : E.cy)));
            } else {
                const int i = lane == 14 ? 7 : lane - 6;
                if (i < 4)
                    v = (top && by == 0) ? 127 : (by > 0 ? s.rec[(ys - 1) * 16 + xs + i] : E.ay[xs + i]);
                else if (by > 0 && bx < 3)
                    v = s.rec[(ys - 1) * 16 + xs + i];
                else if (top)
                    v = 127;
                else if (bx < 3)
                    v = E.ay[xs + i];
                else
                    v = E.ay[15];  // (the right column: only at the frame's right edge may a mode read it)
            }
            B.X[lane] = v;
        }
        wave_lds_sync();
        int pred;
        if (bm == kBDc) {
            pred = (B.X[6] + B.X[7] + B.X[8] + B.X[9] + B.X[1] + B.X[2] + B.X[3] + B.X[4] + 4) >> 3;
        } else if (bm == kBTm) {
            pred = v8_clamp255(B.X[4 - r] + B.X[6 + c] - B.X[5]);
        } else {
            const int t = (int)(((bm < 6 ? taplo >> (8 * (bm - 2)) : taphi >> (8 * (bm - 6)))) & 0xffu), k = t & 15;
            pred = (t & 16) ? (B.X[k] + 2 * B.X[k + 1] + B.X[k + 2] + 2) >> 2 : (B.X[k] + B.X[k + 1] + 1) >> 1;
        }
        const int res = (int)s.src[(ys + r) * 16 + xs + c] - pred;
        // forward DCT (vp8_core.h fdct4x4): rows, then columns
        int t;
        {
            const int i0 = qbc<0>(res), i1 = qbc<1>(res), i2 = qbc<2>(res), i3 = qbc<3>(res);
            const int a1 = (i0 + i3) * 8, b1 = (i1 + i2) * 8, c1 = (i1 - i2) * 8, d1 = (i0 - i3) * 8;
            const int o0 = a1 + b1, o2 = a1 - b1, o1 = (c1 * 2217 + d1 * 5352 + 14500) >> 12,
                      o3 = (d1 * 2217 - c1 * 5352 + 7500) >> 12;
            t = pick4(c, o0, o1, o2, o3);
        }
        int co;
        {
            int tc[4];
            col4(t, r, tc);
            const int a1 = tc[0] + tc[3], b1 = tc[1] + tc[2], c1 = tc[1] - tc[2], d1 = tc[0] - tc[3];
            const int o0 = (a1 + b1 + 7) >> 4, o2 = (a1 - b1 + 7) >> 4;
            const int o1 = ((c1 * 2217 + d1 * 5352 + 12000) >> 16) + (d1 != 0 ? 1 : 0);
            const int o3 = (d1 * 2217 - c1 * 5352 + 51000) >> 16;
            co = pick4(r, o0, o1, o2, o3);
        }
        // quantiser (type 3: the DC at Y1 DC), levels in scan order
        const int qs = q == 0 ? qdc : qac;
        const int lvl = qz(co, qs, q == 0 ? mdc : mac);
        if (lane < 16) lv[b * 16 + kq] = (int16_t)lvl;
        if (__ballot(lane < 16 && lvl != 0)) nz |= 1u << b;
        const int dq = lvl * qs;
        // inverse DCT (vp8_core.h idct4x4): columns, then rows
        constexpr int c8 = 20091, s8 = 35468;
        int u;
        {
            int ic[4];
            col4(dq, r, ic);
            const int a1 = ic[0] + ic[2], b1 = ic[0] - ic[2];
            const int c1 = ((ic[1] * s8) >> 16) - (ic[3] + ((ic[3] * c8) >> 16));
            const int d1 = (ic[1] + ((ic[1] * c8) >> 16)) + ((ic[3] * s8) >> 16);
            u = pick4(r, a1 + d1, b1 + c1, b1 - c1, a1 - d1);
        }
        {
            const int p0 = qbc<0>(u), p1 = qbc<1>(u), p2 = qbc<2>(u), p3 = qbc<3>(u);
            const int a1 = p0 + p2, b1 = p0 - p2;
            const int c1 = ((p1 * s8) >> 16) - (p3 + ((p3 * c8) >> 16));
            const int d1 = (p1 + ((p1 * c8) >> 16)) + ((p3 * s8) >> 16);
            const int o = pick4(c, (a1 + d1 + 4) >> 3, (b1 + c1 + 4) >> 3, (b1 - c1 + 4) >> 3, (a1 - d1 + 4) >> 3);
            if (lane < 16) s.rec[(ys + r) * 16 + xs + c] = (uint8_t)v8_clamp255(pred + o);
        }
        wave_lds_sync();
    }
    return nz;
}

// B_PRED plans of every macroblock of a key frame (vp8_core.h bpred_plan), one wave per
// macroblock, ahead of the k_vp8_key wavefront: the source footprint staged in LDS, lane
// 4 b + r = sub-block b, sample row r, the ten modes in turn; the plan goes into the record
// (ymode kBPred or 0, the modes in the vector words and bmodes_hi), which k_vp8_key reads
// before it writes the macroblock's final record.
__global__ __launch_bounds__(256) void k_vp8_bpred_plan(h264::Geometry g, const Vp8States* __restrict__ st,
                                                        const uint8_t* __restrict__ src_y, Vp8Mb* __restrict__ mbs) {
    __shared__ int Xs[4][16][16];
    __shared__ uint8_t tile[4][17][21];  // rows y0 - 1 .. y0 + 15, columns x0 - 1 .. x0 + 19
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mbi = blockIdx.x * 4 + wave;
    if (mbi >= g.mb_w * g.mb_h) return;  // (wave-uniform; wave-level LDS ordering only below)
    const Vp8FrameState& F = st->v;
    const int lam = F.bpred_lambda;
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w, x0 = mbx * 16, y0 = mby * 16;
    for (int i = lane; i < 17 * 21; i += 64) {
        const int rr = i / 21, cc = i - rr * 21, x = x0 - 1 + cc, y = y0 - 1 + rr;
        tile[wave][rr][cc] = (x >= 0 && y >= 0 && x < g.coded_w) ? src_y[(size_t)y * g.pitch + x] : 0;
    }
    wave_lds_sync();
    auto src = [&](int x, int y) { return (int)tile[wave][y - y0 + 1][x - x0 + 1]; };
    const int b = lane >> 2, rr = lane & 3, bx = b & 3, by = b >> 2;
    if (rr == 0) {
        int X[15];
        bpred_edge(sub_edge(src, mbx, mby, g.mb_w, bx, by), X);
#pragma unroll
        for (int i = 0; i < 15; ++i) Xs[wave][b][i] = X[i];
    }
    // 16x16 modes (lane: row lane / 4, columns 4 (lane % 4) .. + 3)
    const bool at = y0 > 0, al = x0 > 0;
    const int r16 = lane >> 2, c4 = (lane & 3) * 4;
    const int corner = !at ? 127 : (!al ? 129 : src(x0 - 1, y0 - 1));
    const int lft = al ? src(x0 - 1, y0 + r16) : 129;
    const int dcy = dc_value(wsum((lane < 16 && at ? src(x0 + lane, y0 - 1) : 0) + (lane >= 16 && lane < 32 && al ? src(x0 - 1, y0 + lane - 16) : 0)),
                             (at ? 1 : 0) + (al ? 1 : 0), 3);
    uint32_t cost16 = ~0u;
    {
        int sad[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int sv = src(x0 + c4 + j, y0 + r16), abv = at ? src(x0 + c4 + j, y0 - 1) : 127;
#pragma unroll
            for (int m = 0; m < 4; ++m) sad[m] += abs(sv - pred_of(m, abv, lft, corner, dcy));
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t cst = 256u * (uint32_t)wsum(sad[m]) + (uint32_t)(lam * kf_ymode_cost256(m));
            cost16 = cst < cost16 ? cst : cost16;
        }
    }
    wave_lds_sync();
    // sub-block modes
    uint32_t best = ~0u;
    int bm = kBDc;
    const int* X = Xs[wave][b];
    for (int m = 0; m < kNumBModes; ++m) {
        int sad = 0;
#pragma unroll
        for (int x = 0; x < 4; ++x) sad += abs(src(x0 + bx * 4 + x, y0 + by * 4 + rr) - bpred_px(m, X, x, rr));
        sad += __builtin_amdgcn_mov_dpp(sad, 0xB1, 0xF, 0xF, false);
        sad += __builtin_amdgcn_mov_dpp(sad, 0x4E, 0xF, 0xF, false);
        const uint32_t cst = 256u * (uint32_t)sad + (uint32_t)(lam * bmode_plan_cost256(m));
        if (bmode_allowed(m, bx, mbx, mby, g.mb_w) && cst < best) {
            best = cst;
            bm = m;
        }
    }
    const uint32_t costb = (uint32_t)(lam * kf_ymode_cost256(kBPred)) + (uint32_t)wsum(rr == 0 ? (int)best : 0);
    const uint32_t lo = (uint32_t)wsum(rr == 0 && b < 8 ? (int)((uint32_t)bm << (4 * b)) : 0);
    const uint32_t hi = (uint32_t)wsum(rr == 0 && b >= 8 ? (int)((uint32_t)bm << (4 * (b - 8))) : 0);
    if (lane == 0) {
        Vp8Mb& m = mbs[mbi];
        m.mvx = (int16_t)(uint16_t)(lo & 0xffffu);
        m.mvy = (int16_t)(uint16_t)(lo >> 16);
        m.ymode = (uint8_t)(costb < cost16 ? kBPred : 0);
        m.bmodes_hi = hi;
    }
}

__global__ __launch_bounds__(64) void k_vp8_key(h264::Geometry g, const Vp8States* __restrict__ st,
                                                 const uint8_t* __restrict__ src_y,
                                                 const uint8_t* __restrict__ src_uv, Vp8Mb* __restrict__ mbs,
                                                 int16_t* __restrict__ lv,
                                                 uint64_t* __restrict__ line, int* __restrict__ err) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    __shared__ MbLds s;
    __shared__ KeyEdges E;
    __shared__ BpLds B;
    const Vp8FrameState& F = st->v;
    const int mby = blockIdx.x, lane = threadIdx.x, y0 = mby * 16;
    const uint32_t epoch = (uint32_t)F.epoch;
    const bool top = mby == 0, bottom = mby == g.mb_h - 1;
    // hand-off words of a macroblock: 0..3 its bottom luma row, 4..7 its bottom chroma row
    // (interleaved), 32 samples each with the frame's epoch tag above them
    constexpr int W = kKeyLineWords;
    const uint64_t* above_line = line + (size_t)(mby > 0 ? mby - 1 : 0) * g.mb_w * W;
    uint64_t* my_line = line + (size_t)mby * g.mb_w * W;
    // the source of the next macroblock is fetched one macroblock ahead (registers), staged in LDS
    // at the top of the iteration; the fetch is taken at the bottom of the iteration that issued
    // it, so its wait counts the stores after it, not a vmcnt(0) at the loop's join
    const int sr = lane >> 2, sc4 = (lane & 3) * 4;
    // ... and so is its B_PRED plan (k_vp8_bpred_plan: the record's vector words, ymode, bmodes_hi)
    const bool bpred = F.bpred_lambda != 0;
    auto fetch = [&](int x0n, uint32_t& wy, uint32_t& wuv, uint4& pl) {
        wy = *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y0 + sr) * g.pitch + x0n + sc4);
        wuv = *reinterpret_cast<const uint32_t*>(src_uv + (size_t)(y0 / 2 + (sr & 7)) * g.pitch + x0n + sc4);
        if (bpred) {
            const uint32_t* pw = reinterpret_cast<const uint32_t*>(mbs + mby * g.mb_w + x0n / 16);
            pl = make_uint4(pw[0], pw[1], pw[7], 0u);
        }
    };
    uint32_t nwy, nwuv;
    uint4 npl = make_uint4(0u, 0u, 0u, 0u);
    fetch(0, nwy, nwuv, npl);
    // kBPredTap of this lane's sample (lane % 16) for the eight table modes, a byte each
    uint32_t taplo = 0, taphi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        taplo |= (uint32_t)kBPredTap[k][lane & 15] << (8 * k);
        taphi |= (uint32_t)kBPredTap[4 + k][lane & 15] << (8 * k);
    }
    // the finished macroblock's reconstruction words and record, stored one macroblock late (after
    // the next poll, whose vmcnt(0) would otherwise wait for these stores)
    uint32_t pwy = 0, pwuv = 0, psse[3] = {0, 0, 0};
    int pmbx = -1, pym = 0, puvm = 0;
    uint32_t pnz = 0, pblo = 0, pbhi = 0;
    auto flush = [&]() {
        if (pmbx < 0) return;
        const int r = lane >> 2, c4 = (lane & 3) * 4, px0 = pmbx * 16;
        *reinterpret_cast<uint32_t*>(F.rec_y + (size_t)(y0 + r) * g.pitch + px0 + c4) = pwy;
        if (lane < 32) *reinterpret_cast<uint32_t*>(F.rec_uv + (size_t)(y0 / 2 + r) * g.pitch + px0 + c4) = pwuv;
        store_record(mbs + mby * g.mb_w + pmbx, (int)(int16_t)(pblo & 0xffffu), (int)(int16_t)(pblo >> 16), pym, puvm,
                     pnz, psse, lane, 0, pbhi);
        pmbx = -1;
    };
    for (int mbx = 0; mbx < g.mb_w; ++mbx) {
        const int x0 = mbx * 16, mbi = mby * g.mb_w + mbx;
        const bool left = mbx > 0;
        {  // stage_src from the fetched words
            *reinterpret_cast<uint32_t*>(s.src + sr * 16 + sc4) = nwy;
            if (lane < 32) {
                const int o = sr * 8 + (sc4 >> 1);
                s.su[o] = (uint8_t)nwuv;  // U V U V
                s.sv[o] = (uint8_t)(nwuv >> 8);
                s.su[o + 1] = (uint8_t)(nwuv >> 16);
                s.sv[o + 1] = (uint8_t)(nwuv >> 24);
            }
        }
        // ---- edges: above row and corner from the row above (hand-off line), left from our last MB
        if (!top) {
            // the row above's words of this macroblock (lanes 0..7) and of the one before it (lanes
            // 8, 9: the corner samples), polled until every needed word carries this frame's tag
            // (tagged 64-bit agent-scope atomics: no release fence -- an L2 write-back -- per MB)
            const bool need = lane < 8 || (lane < 10 && left);
            const int wi = lane < 8 ? W * mbx + lane : W * (mbx - 1) + (lane == 8 ? 3 : 7);
            const gu64* wp = (const gu64*)(above_line + (need ? wi : 0));
            uint64_t w = 0;
            for (unsigned sp = 0;; ++sp) {
                w = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!__any(need && (uint32_t)(w >> 32) != epoch)) break;
                if (sp > kSpinLimit) {
                    *err = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            const uint32_t d = (uint32_t)w;
            if (lane < 4) {
#pragma unroll
                for (int k = 0; k < 4; ++k) E.ay[4 * lane + k] = (int)((d >> (8 * k)) & 0xff);
            } else if (lane < 8) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    E.au[2 * (lane - 4) + k] = (int)((d >> (16 * k)) & 0xff);
                    E.av[2 * (lane - 4) + k] = (int)((d >> (16 * k + 8)) & 0xff);
                }
            } else if (lane == 8) {
                E.cy = left ? (int)(d >> 24) : 129;
            } else if (lane == 9) {
                E.cu = left ? (int)((d >> 16) & 0xff) : 129;
                E.cv = left ? (int)(d >> 24) : 129;
            }
        } else {
            if (lane < 16) E.ay[lane] = 127;
            if (lane < 8) E.au[lane] = E.av[lane] = 127;
            if (lane == 0) E.cy = E.cu = E.cv = 127;
        }
        if (!left) {
            if (lane < 16) E.ly[lane] = 129;
            if (lane < 8) E.lu[lane] = E.lvv[lane] = 129;
        }
        // this macroblock's plan (wave-uniform), then the next macroblock's fetch
        const bool bp = bpred && (npl.y & 0xffu) == kBPred;
        const uint32_t blo = bp ? npl.x : 0u, bhi = bp ? npl.z : 0u;
        fetch(mbx + 1 < g.mb_w ? x0 + 16 : x0, nwy, nwuv, npl);  // (after the poll: its waits drain all loads)
        flush();  // the previous macroblock's reconstruction and record (after the poll, likewise)
        __syncthreads();
        // ---- mode decisions: SAD of the four 16x16 modes (4 samples per lane), the four chroma modes
        const int nav = top ? 0 : 1, nlf = left ? 1 : 0;
        const int dcy = dc_value(wsum((lane < 16 && !top ? E.ay[lane] : 0) + (lane >= 16 && lane < 32 && left ? E.ly[lane - 16] : 0)),
                                 nav + nlf, 3);
        const int dcu = dc_value(wsum((lane < 8 && !top ? E.au[lane] : 0) + (lane >= 8 && lane < 16 && left ? E.lu[lane - 8] : 0)),
                                 nav + nlf, 2);
        const int dcv = dc_value(wsum((lane < 8 && !top ? E.av[lane] : 0) + (lane >= 8 && lane < 16 && left ? E.lvv[lane - 8] : 0)),
                                 nav + nlf, 2);
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        int ymode = 0, uvmode = 0;
        if (!bp) {
            uint32_t best16 = ~0u;
            int sad[4] = {0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int sv = s.src[r * 16 + c4 + j];
#pragma unroll
                for (int m = 0; m < 4; ++m) sad[m] += abs(sv - pred_of(m, E.ay[c4 + j], E.ly[r], E.cy, dcy));
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t t = (uint32_t)wsum(sad[m]);
                if (t < best16) {
                    best16 = t;
                    ymode = m;
                }
            }
        }
        const int cx = lane & 7, cy = lane >> 3;
        {
            int sad[4] = {0, 0, 0, 0};
            const int su = s.su[cy * 8 + cx], sv = s.sv[cy * 8 + cx];
#pragma unroll
            for (int m = 0; m < 4; ++m)
                sad[m] = abs(su - pred_of(m, E.au[cx], E.lu[cy], E.cu, dcu)) +
                         abs(sv - pred_of(m, E.av[cx], E.lvv[cy], E.cv, dcv));
            uint32_t best = ~0u;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t t = (uint32_t)wsum(sad[m]);
                if (t < best) {
                    best = t;
                    uvmode = m;
                }
            }
        }
        if (!bp)
#pragma unroll
            for (int j = 0; j < 4; ++j) s.pred[r * 16 + c4 + j] = (uint8_t)pred_of(ymode, E.ay[c4 + j], E.ly[r], E.cy, dcy);
        s.pu[cy * 8 + cx] = (uint8_t)pred_of(uvmode, E.au[cx], E.lu[cy], E.cu, dcu);
        s.pv[cy * 8 + cx] = (uint8_t)pred_of(uvmode, E.av[cx], E.lvv[cy], E.cv, dcv);
        __syncthreads();
        // ---- B_PRED (planned): the sub-blocks coded in turn into s.rec, then the chroma
        uint32_t bnz = 0;
        if (bp) {
            bnz = bpred_code_gpu(s, B, E, F, lv + (size_t)mbi * kCoefPerMb, lane, mbx, mby, blo, bhi, taplo, taphi);
            ymode = kBPred;
            __syncthreads();
        }
        const uint32_t nz = code_mb(s, F, lv + (size_t)mbi * kCoefPerMb, lane, -1, 0, bp) | bnz;
        // ---- hand the bottom rows down: eight tagged words
        if (!bottom && lane < W) {
            uint32_t d = 0;
            if (lane < 4) {
#pragma unroll
                for (int k = 0; k < 4; ++k) d |= (uint32_t)s.rec[15 * 16 + 4 * lane + k] << (8 * k);
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    d |= ((uint32_t)s.ru[7 * 8 + 2 * (lane - 4) + k] << (16 * k)) |
                         ((uint32_t)s.rv[7 * 8 + 2 * (lane - 4) + k] << (16 * k + 8));
            }
            __hip_atomic_store((gu64*)(my_line + W * mbx + lane), (uint64_t)d | ((uint64_t)epoch << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        rec_words(s, g, x0, y0, lane, pwy, pwuv, psse);
        pmbx = mbx;
        pym = ymode;
        puvm = uvmode;
        pnz = nz;
        pblo = blo;
        pbhi = bhi;
        // left edges of the next macroblock
        if (lane < 16) E.ly[lane] = s.rec[lane * 16 + 15];
        if (lane < 8) {
            E.lu[lane] = s.ru[lane * 8 + 7];
            E.lvv[lane] = s.rv[lane * 8 + 7];
        }
        asm volatile("" : "+v"(nwy), "+v"(nwuv), "+v"(npl.x), "+v"(npl.y), "+v"(npl.z));  // fetched a macroblock ago
        __syncthreads();
    }
    flush();
}

// ------------------------------------------------------------------ intra macroblocks in P frames
// vp8_core.h vp8_intra_candidate, CpuVp8Encoder::intra_pass: two fully parallel passes after
// k_vp8_inter (one wave per macroblock each).  Edges of a macroblock from the frame's
// reconstruction with VP8's frame-edge values (lanes 0..15 luma row / column, 16..23 the chroma
// rows, 24..31 the chroma columns, 32 the corners).
__device__ __forceinline__ void rec_edges(KeyEdges& E, const h264::Geometry& g, const Vp8FrameState& F, int x0, int y0,
                                          int lane) {
    const bool top = y0 == 0, left = x0 > 0;
    const size_t P = g.pitch;
    if (lane < 16) {
        E.ay[lane] = top ? 127 : F.rec_y[(size_t)(y0 - 1) * P + x0 + lane];
        E.ly[lane] = left ? F.rec_y[(size_t)(y0 + lane) * P + x0 - 1] : 129;
    } else if (lane < 24) {
        const int k = lane - 16;
        E.au[k] = top ? 127 : F.rec_uv[(size_t)(y0 / 2 - 1) * P + x0 + 2 * k];
        E.av[k] = top ? 127 : F.rec_uv[(size_t)(y0 / 2 - 1) * P + x0 + 2 * k + 1];
    } else if (lane < 32) {
        const int k = lane - 24;
        E.lu[k] = left ? F.rec_uv[(size_t)(y0 / 2 + k) * P + x0 - 2] : 129;
        E.lvv[k] = left ? F.rec_uv[(size_t)(y0 / 2 + k) * P + x0 - 1] : 129;
    } else if (lane == 32) {
        E.cy = top ? 127 : (!left ? 129 : F.rec_y[(size_t)(y0 - 1) * P + x0 - 1]);
        E.cu = top ? 127 : (!left ? 129 : F.rec_uv[(size_t)(y0 / 2 - 1) * P + x0 - 2]);
        E.cv = top ? 127 : (!left ? 129 : F.rec_uv[(size_t)(y0 / 2 - 1) * P + x0 - 1]);
    }
}

// 16x16 luma mode of least SAD against the staged source (ties: the lower mode), its SAD
__device__ __forceinline__ int best_luma16(const MbLds& s, const KeyEdges& E, bool top, bool left, int lane,
                                           uint32_t& best) {
    const int dcy = dc_value(wsum((lane < 16 && !top ? E.ay[lane] : 0) + (lane >= 16 && lane < 32 && left ? E.ly[lane - 16] : 0)),
                             (top ? 0 : 1) + (left ? 1 : 0), 3);
    const int r = lane >> 2, c4 = (lane & 3) * 4;
    int sad[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int sv = s.src[r * 16 + c4 + j];
#pragma unroll
        for (int m = 0; m < 4; ++m) sad[m] += abs(sv - pred_of(m, E.ay[c4 + j], E.ly[r], E.cy, dcy));
    }
    int mode = 0;
    best = ~0u;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint32_t t = (uint32_t)wsum(sad[m]);
        if (t < best) {
            best = t;
            mode = m;
        }
    }
    return mode;
}

// candidates: one wave per macroblock, four per workgroup (most macroblocks leave at once: the
// inter prediction is good); a candidate appends itself to ilist (ilist[0] = the count, reset by
// k_vp8_inter)
__global__ __launch_bounds__(256) void k_vp8_intra_cand(h264::Geometry g, const Vp8States* __restrict__ st,
                                                         const uint8_t* __restrict__ src_y,
                                                         const uint8_t* __restrict__ src_uv,
                                                         const Vp8Mb* __restrict__ mbs, uint8_t* __restrict__ icand,
                                                         int* __restrict__ ilist) {
    __shared__ MbLds sh[4];
    __shared__ KeyEdges Eh[4];
    const Vp8FrameState& F = st->v;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mbi = blockIdx.x * 4 + wave;
    if (mbi >= g.mb_w * g.mb_h) return;  // (wave-uniform; wave-level LDS ordering only below)
    MbLds& s = sh[wave];
    KeyEdges& E = Eh[wave];
    const uint32_t psad = mbs[mbi].bmodes_hi;
    if (psad <= kIntraMinSad) {
        if (lane == 0) icand[mbi] = 0;
        return;
    }
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w, x0 = mbx * 16, y0 = mby * 16;
    stage_src(s, g, src_y, src_uv, x0, y0, lane);
    rec_edges(E, g, F, x0, y0, lane);
    wave_lds_sync();
    uint32_t best;
    const int mode = best_luma16(s, E, mby == 0, mbx > 0, lane, best);
    const bool cand = vp8_intra_candidate(psad, best, F.intra_lambda);
    if (lane == 0) {
        icand[mbi] = (uint8_t)((cand ? 0x80 : 0) | mode);
        if (cand) ilist[1 + atomicAdd(&ilist[0], 1)] = mbi;
    }
}

// the candidates without a candidate causal neighbour, coded intra: a fixed grid over the
// candidate list (a few percent of the macroblocks at most), one macroblock per workgroup step
constexpr int kIntraCodeGrid = 1024;
__global__ __launch_bounds__(64) void k_vp8_intra_code(h264::Geometry g, const Vp8States* __restrict__ st,
                                                        const uint8_t* __restrict__ src_y,
                                                        const uint8_t* __restrict__ src_uv, Vp8Mb* __restrict__ mbs,
                                                        int16_t* __restrict__ lv, const uint8_t* __restrict__ icand,
                                                        const int* __restrict__ ilist) {
    __shared__ MbLds s;
    __shared__ KeyEdges E;
    const Vp8FrameState& F = st->v;
    const int lane = threadIdx.x;
    const int n = ilist[0];
    for (int li = blockIdx.x; li < n; li += gridDim.x) {
    const int mbi = ilist[1 + li];
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w, x0 = mbx * 16, y0 = mby * 16;
    const int ic = icand[mbi];
    // a candidate without a candidate causal neighbour (workgroup-uniform)
    if ((mbx > 0 && (icand[mbi - 1] & 0x80)) || (mby > 0 && (icand[mbi - g.mb_w] & 0x80)) ||
        (mbx > 0 && mby > 0 && (icand[mbi - g.mb_w - 1] & 0x80)))
        continue;
    const int seg = mbs[mbi].seg;
    stage_src(s, g, src_y, src_uv, x0, y0, lane);
    rec_edges(E, g, F, x0, y0, lane);
    __syncthreads();
    const bool top = mby == 0, left = mbx > 0;
    const int ymode = ic & 3;
    const int nav = top ? 0 : 1, nlf = left ? 1 : 0;
    const int dcy = dc_value(wsum((lane < 16 && !top ? E.ay[lane] : 0) + (lane >= 16 && lane < 32 && left ? E.ly[lane - 16] : 0)),
                             nav + nlf, 3);
    const int dcu = dc_value(wsum((lane < 8 && !top ? E.au[lane] : 0) + (lane >= 8 && lane < 16 && left ? E.lu[lane - 8] : 0)),
                             nav + nlf, 2);
    const int dcv = dc_value(wsum((lane < 8 && !top ? E.av[lane] : 0) + (lane >= 8 && lane < 16 && left ? E.lvv[lane - 8] : 0)),
                             nav + nlf, 2);
    const int r = lane >> 2, c4 = (lane & 3) * 4, cx = lane & 7, cy = lane >> 3;
    int uvmode = 0;
    {
        int sad[4];
        const int su = s.su[cy * 8 + cx], sv = s.sv[cy * 8 + cx];
#pragma unroll
        for (int m = 0; m < 4; ++m)
            sad[m] = abs(su - pred_of(m, E.au[cx], E.lu[cy], E.cu, dcu)) + abs(sv - pred_of(m, E.av[cx], E.lvv[cy], E.cv, dcv));
        uint32_t best = ~0u;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t t = (uint32_t)wsum(sad[m]);
            if (t < best) {
                best = t;
                uvmode = m;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s.pred[r * 16 + c4 + j] = (uint8_t)pred_of(ymode, E.ay[c4 + j], E.ly[r], E.cy, dcy);
    s.pu[cy * 8 + cx] = (uint8_t)pred_of(uvmode, E.au[cx], E.lu[cy], E.cu, dcu);
    s.pv[cy * 8 + cx] = (uint8_t)pred_of(uvmode, E.av[cx], E.lvv[cy], E.cv, dcv);
    __syncthreads();
    const uint32_t nz = code_mb(s, F, lv + (size_t)mbi * kCoefPerMb, lane, -1, seg);
    uint32_t sse[3];
    store_rec(s, g, F, x0, y0, lane, sse);
    store_record(mbs + mbi, 0, 0, ymode, uvmode, nz, sse, lane, seg, 0);
    __syncthreads();  // (LDS reuse by the next list entry)
    }
}

// ------------------------------------------------------------------ loop filter (15)
// The whole reconstruction in place, bit-exact with vp8_core.h loop_filter_frame.  Section 15.1 is
// a raster-order chain: a macroblock's left edge reads the columns its left neighbour's inner and
// horizontal edges left, its top edge the rows the row above left after that row's next
// macroblock filtered its left edge.  So: one wave per macroblock row walking the row, the row
// below two macroblocks behind; kLfRows rows per workgroup.  Lanes 0..15 own luma lines, 16..23
// Cb, 24..31 Cr: the vertical edges run on sample rows in registers (elements 0..3 the left
// neighbour's last four columns, 4.. the macroblock), the horizontal edges on columns after a
// transpose through the wave's LDS tile (elements 0..3 the four rows above).
// Hand-offs: inside a workgroup a row passes each finished macroblock's bottom rows 12..15 to the
// row below through an LDS ring (progress words, back-pressure at kLfRing entries); across
// workgroups (other XCDs, other L2s) the last row stores the same rows, column-packed, into a
// hand-off line of 64-bit words -- four samples and the frame's epoch tag -- with agent-scope
// atomic stores (device-coherent: no L2 write-back fence, no separate progress word to order
// after them); the next workgroup's first row polls its words with agent-scope atomic loads until
// every lane holds this frame's tag.  Every
// sample has one writer: a row writes rows 0..12 of its macroblock x - 1 once x's left edge is
// done; rows 13..15 go out with the row below's top-edge strip.  The distortion against the
// source of every final sample is summed per row (the frame statistics; the records' figures are
// the unfiltered picture's).  The macroblocks' levels and inner-edge flags are staged in LDS
// first.  Global accesses go through address-space-1 pointers (flat ones would also count on
// lgkmcnt and stall every LDS wait); the transposes order LDS with compiler barriers only (a
// wave's LDS operations execute in order; a fence would wait for the prefetched loads).
constexpr int kLfRows = 4;  // one wave per SIMD (8 rows, two per SIMD, measured 5 % slower)
constexpr int kLfRing = 8;
struct LfWave {
    uint8_t T[512];                // transposes: luma 16x16 at 0, Cb 8x8 at 256, Cr 8x8 at 320
    uint8_t ring[kLfRing][128];    // rows 12..15 of a macroblock: luma 4 x 16, then chroma 4 x 16 interleaved
    uint8_t info[512];             // per macroblock of the row: level | inner-edges << 7
    int prod;                      // ring entries written (macroblocks 0 .. prod - 1)
    int cons;                      // entries of the row above's ring this row has read
};
typedef __attribute__((address_space(1))) uint8_t g8;
typedef unsigned LfV4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) LfV4 GLfV4;
__device__ __forceinline__ uint4 lf_ld16(const uint8_t* p) {
    const LfV4 v = *(const GLfV4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lf_st16(uint8_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const LfV4 v = {a, b, c, d};
    *(GLfV4*)p = v;
}
__device__ __forceinline__ uint32_t byte_of(const uint4& w, int j) {
    const uint32_t d = j < 4 ? w.x : (j < 8 ? w.y : (j < 12 ? w.z : w.w));
    return (d >> (8 * (j & 3))) & 0xffu;
}
__device__ __forceinline__ void lf_sync_wave() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ int lf_lds_load(const int* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}
__device__ __forceinline__ void lf_lds_store(int* p, int v) {  // LDS writes before it visible first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lf_wait_lds(const int* p, int need, int* err) {
    for (unsigned s = 0; lf_lds_load(p) < need; ++s) {
        if (s > kSpinLimit) {
            *err = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Lanes 32..63 mirror lanes 0..31 (same loads, same values, same stores): every vector memory
// instruction of the loop then runs unconditionally (no lane-divergent branch around it), so the
// compiler's vmcnt wait for the prefetched row counts only the operations issued after it instead
// of falling back to vmcnt(0) at a join -- which drained the prefetch and the stores.  Stores a
// lane must not make (rows 13..15, Cr lanes' halves) go to the wave's scratch words.  The
// distortion of the filtered picture is k_vp8_lf_sse's (fully parallel, off this chain).
template <int kRows>
__global__ __launch_bounds__(64 * kRows) void k_vp8_lf(h264::Geometry g, const Vp8States* __restrict__ st,
                                                        const Vp8Mb* __restrict__ mbs,
                                                        unsigned long long* __restrict__ line,
                                                        int* __restrict__ err) {
    __builtin_amdgcn_s_setprio(3);  // a serial chain on few waves
    __shared__ LfWave W[kRows];
    const int wr = threadIdx.x >> 6, lane = threadIdx.x & 63, ml = lane & 31;
    const int mby = blockIdx.x * kRows + wr;
    if (threadIdx.x < kRows) W[threadIdx.x].prod = W[threadIdx.x].cons = 0;
    __syncthreads();
    if (mby >= g.mb_h) return;
    const Vp8FrameState& F = st->v;
    LfWave& S = W[wr];
    const int y0 = mby * 16, cy0 = mby * 8;
    const uint32_t epoch = (uint32_t)F.epoch;
    const bool is_y = ml < 16, is_u = ml >= 16 && ml < 24;
    const int li = is_y ? ml : (ml - 16) & 7;  // the lane's line (row, then column) of its plane
    const int comp = is_u ? 0 : 1;             // chroma component byte in an interleaved pair
    const int pitch = g.pitch;
    const bool bottom = mby == g.mb_h - 1;
    const bool wg_last = wr == kRows - 1 && !bottom;  // hands off to the next workgroup
    const bool ring_out = wr < kRows - 1 && !bottom;  // hands off to the next wave
    const bool glb_in = wr == 0 && mby > 0;            // rows above from the previous workgroup
    const bool key = F.key != 0;
    uint8_t* const rec_y = F.rec_y;
    uint8_t* const rec_uv = F.rec_uv;
    const size_t line_words = (size_t)32 * g.mb_w * (size_t)((g.mb_h + kRows - 1) / kRows);  // 64-bit
    uint8_t* const scratch = reinterpret_cast<uint8_t*>(line + line_words) + (size_t)(blockIdx.x * kRows + wr) * 1024;
    // row-phase line of this lane (luma row li / chroma row li, interleaved)
    uint8_t* const rrow = is_y ? rec_y + (size_t)(y0 + li) * pitch : rec_uv + (size_t)(cy0 + li) * pitch;
    // column-phase sample (x0 + col) of row y0 - 4 + k of this lane's plane: byte offset
    auto col_off = [&](int x0, int k) -> size_t {
        return is_y ? (size_t)(y0 - 4 + k) * pitch + x0 + li : (size_t)(cy0 - 4 + k) * pitch + x0 + 2 * li + comp;
    };
    uint8_t* const cplane = is_y ? rec_y : rec_uv;
    // transposes: luma 16x16 at T + 0 (row-major), Cb / Cr 8x8 at 256 / 320
    const int tb = is_y ? 0 : (is_u ? 256 : 320), tstride = is_y ? 16 : 8;
    // rows this lane writes back: rows 13..15 (chroma 5..7) belong to the row below's strip; a Cr
    // lane's samples go out interleaved by its Cb lane
    const bool writes_row = (is_y || is_u) && (bottom || (is_y ? li <= 12 : li <= 4));
    // stage the row's macroblock levels and inner-edge flags
    for (int i = lane; i < g.mb_w; i += 64) {
        const Vp8Mb& m = mbs[mby * g.mb_w + i];
        S.info[i] = (uint8_t)(F.lf_level[m.seg & 3] | ((m.nz || m.ymode == kBPred) ? 0x80 : 0));  // B_PRED: inner edges always
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the staged bytes before any lane reads them
    lf_sync_wave();
    int px[20], fin[16];
#pragma unroll
    for (int j = 0; j < 20; ++j) px[j] = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) fin[j] = 0;
    uint4 own = lf_ld16(rrow);  // macroblock 0's row
    int cons_seen = 0;          // the row below's ring progress last read (back-pressure)
    // the first row of a workgroup: line word of the next macroblock, loaded a step ahead (other
    // rows load their scratch: the same instruction stream) -- a workgroup boundary then costs one
    // hand-off latency once, not a global round trip every step
    const unsigned long long* const line_in =
        glb_in ? line + ((size_t)(blockIdx.x - 1) * g.mb_w) * 32 + ml : reinterpret_cast<const unsigned long long*>(scratch) + 64 + ml;
    const int line_step = glb_in ? 32 : 0;
    uint64_t pre = __hip_atomic_load((const gu64*)line_in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto pack4 = [&](int k) -> uint32_t {
        return (uint32_t)fin[4 * k] | ((uint32_t)fin[4 * k + 1] << 8) | ((uint32_t)fin[4 * k + 2] << 16) |
               ((uint32_t)fin[4 * k + 3] << 24);
    };
    auto store_mb = [&](int mbx_done) {
        uint32_t d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = pack4(k);
        // Cr lanes hand their 8 samples to the Cb lane of the same row: DPP row_ror:8 (lane l of a
        // 16-lane row reads lane l ^ 8)
        const uint32_t vlo = (uint32_t)__builtin_amdgcn_mov_dpp((int)d[0], 0x128, 0xF, 0xF, false);
        const uint32_t vhi = (uint32_t)__builtin_amdgcn_mov_dpp((int)d[1], 0x128, 0xF, 0xF, false);
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t uw = d[k >> 1] >> (16 * (k & 1)), vw = (k < 2 ? vlo : vhi) >> (16 * (k & 1));
            const uint32_t c = (uw & 0xffu) | ((vw & 0xffu) << 8) | (((uw >> 8) & 0xffu) << 16) |
                               (((vw >> 8) & 0xffu) << 24);
            o[k] = is_y ? d[k] : c;
        }
        lf_st16(writes_row ? rrow + mbx_done * 16 : scratch + 16 * lane, o[0], o[1], o[2], o[3]);
    };
    // rows 12..15 (chroma 4..7) of the finished macroblock into the ring for the row below (the
    // workgroup's last row: into the hand-off line for the next workgroup, through its ring entry)
    unsigned long long* const line_out = line + (size_t)blockIdx.x * g.mb_w * 32;
    auto ring_put = [&](int mbx_done) {
        if (!ring_out && !wg_last) return;
        if (ring_out && cons_seen < mbx_done - kLfRing + 1) {  // back-pressure
            lf_wait_lds(&W[wr + 1].cons, mbx_done - kLfRing + 1, err);
            cons_seen = lf_lds_load(&W[wr + 1].cons);
        }
        uint8_t* e = S.ring[mbx_done % kLfRing];
        if (is_y && li >= 12) {
#pragma unroll
            for (int k = 0; k < 4; ++k) *reinterpret_cast<uint32_t*>(e + (li - 12) * 16 + 4 * k) = pack4(k);
        } else if (!is_y && li >= 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j) e[64 + (li - 4) * 16 + 2 * j + comp] = (uint8_t)fin[j];
        }
        if (wg_last) {  // column-packed line word ml: luma column, then Cb, Cr columns
            lf_sync_wave();
            const int o = is_y ? li : 64 + 2 * li + comp;
            const uint32_t w = (uint32_t)e[o] | ((uint32_t)e[o + 16] << 8) | ((uint32_t)e[o + 32] << 16) |
                               ((uint32_t)e[o + 48] << 24);
            __hip_atomic_store((gu64*)(line_out + (size_t)mbx_done * 32 + ml), (uint64_t)w | ((uint64_t)epoch << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lf_sync_wave();
        } else {
            lf_lds_store(&S.prod, mbx_done + 1);
        }
    };
    for (int mbx = 0; mbx < g.mb_w; ++mbx) {
        const int x0 = mbx * 16;
        const int inf = __builtin_amdgcn_readfirstlane((int)S.info[mbx]);
        const int level = inf & 63;  // wave-uniform
        const LfParams f = lf_params(level, key);
        const bool inner = (inf & 0x80) != 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) px[4 + j] = is_y ? (int)byte_of(own, j) : (j < 8 ? (int)byte_of(own, 2 * j + comp) : 0);
        // ---- vertical edges: left macroblock edge, inner edges (luma 4 / 8 / 12, chroma 4)
        if (level) {
            if (mbx > 0) lf_mb_edge(px, f);
            if (inner) {
                lf_sub_edge(px + 4, f);
                if (is_y) {
                    lf_sub_edge(px + 8, f);
                    lf_sub_edge(px + 12, f);
                }
            }
        }
        // macroblock mbx - 1 is final for this row now
        if (mbx > 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (is_y)
                    fin[12 + k] = px[k];
                else
                    fin[4 + k] = px[k];
            }
            ring_put(mbx - 1);
            store_mb(mbx - 1);
        }
        // ---- the four rows above this macroblock (columns)
        int cl[20];
#pragma unroll
        for (int k = 0; k < 20; ++k) cl[k] = 0;
        if (glb_in) {
            uint64_t w = pre;
            if (__any((uint32_t)(w >> 32) != epoch)) {  // not there yet: poll
                const gu64* p = (const gu64*)(line_in + (size_t)mbx * line_step);
                for (unsigned sp = 0;; ++sp) {
                    __builtin_amdgcn_s_sleep(1);
                    w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (!__any((uint32_t)(w >> 32) != epoch)) break;
                    if (sp > kSpinLimit) {
                        *err = 1;
                        break;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) cl[k] = (int)((w >> (8 * k)) & 0xffu);
        } else if (mby > 0) {
            lf_wait_lds(&W[wr - 1].prod, mbx + 1, err);
            const uint8_t* e = W[wr - 1].ring[mbx % kLfRing];
#pragma unroll
            for (int k = 0; k < 4; ++k) cl[k] = (int)e[is_y ? k * 16 + li : 64 + k * 16 + 2 * li + comp];
            lf_lds_store(&S.cons, mbx + 1);  // (waits for the reads above)
        }
        // prefetch the next macroblock's line word and row (unconditional: the waits count exactly)
        pre = __hip_atomic_load((const gu64*)(line_in + (size_t)(mbx + 1 < g.mb_w ? mbx + 1 : mbx) * line_step),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        own = lf_ld16(rrow + (mbx + 1 < g.mb_w ? x0 + 16 : x0));
        if (level) {
            if (is_y) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *reinterpret_cast<uint32_t*>(S.T + li * 16 + 4 * k) =
                        (uint32_t)px[4 + 4 * k] | ((uint32_t)px[5 + 4 * k] << 8) | ((uint32_t)px[6 + 4 * k] << 16) |
                        ((uint32_t)px[7 + 4 * k] << 24);
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    *reinterpret_cast<uint32_t*>(S.T + tb + li * 8 + 4 * k) =
                        (uint32_t)px[4 + 4 * k] | ((uint32_t)px[5 + 4 * k] << 8) | ((uint32_t)px[6 + 4 * k] << 16) |
                        ((uint32_t)px[7 + 4 * k] << 24);
            }
            lf_sync_wave();
#pragma unroll
            for (int r = 0; r < 16; ++r) cl[4 + r] = is_y || r < 8 ? (int)S.T[tb + r * tstride + li] : 0;
            lf_sync_wave();
            if (mby > 0) lf_mb_edge(cl, f);
            if (inner) {
                lf_sub_edge(cl + 4, f);
                if (is_y) {
                    lf_sub_edge(cl + 8, f);
                    lf_sub_edge(cl + 12, f);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (is_y || r < 8) S.T[tb + r * tstride + li] = (uint8_t)cl[4 + r];
            lf_sync_wave();
            if (is_y) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(S.T + li * 16 + 4 * k);
#pragma unroll
                    for (int b = 0; b < 4; ++b) fin[4 * k + b] = (int)((w >> (8 * b)) & 0xffu);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(S.T + tb + li * 8 + 4 * k);
#pragma unroll
                    for (int b = 0; b < 4; ++b) fin[4 * k + b] = (int)((w >> (8 * b)) & 0xffu);
                }
#pragma unroll
                for (int j = 8; j < 16; ++j) fin[j] = 0;
            }
            lf_sync_wave();
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) fin[j] = px[4 + j];
        }
        // the strip above (rows 13..15 of the macroblock above): final now, written back by this
        // row (the row above wrote rows 0..12 only); the top row stores to its scratch words
#pragma unroll
        for (int k = 1; k < 4; ++k) *(g8*)(mby > 0 ? cplane + col_off(x0, k) : scratch + 64 * k + lane) = (uint8_t)cl[k];
        // left context of the next macroblock
#pragma unroll
        for (int k = 0; k < 4; ++k) px[k] = is_y ? fin[12 + k] : fin[4 + k];
        // the prefetched row is taken here, inside the iteration (its wait counts only the strip
        // stores after it; taken at the top of the next iteration, the join with the loop entry
        // made it a full vmcnt(0))
        {
            uint32_t a0 = own.x, a1 = own.y, a2 = own.z, a3 = own.w, p0 = (uint32_t)pre, p1 = (uint32_t)(pre >> 32);
            asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(p0), "+v"(p1));
            own = make_uint4(a0, a1, a2, a3);
            pre = (uint64_t)p0 | ((uint64_t)p1 << 32);
        }
    }
    ring_put(g.mb_w - 1);
    store_mb(g.mb_w - 1);
}

// Distortion of the filtered picture against the source: one workgroup per macroblock row,
// partials per row and channel over the display area (the frame statistics).
__global__ __launch_bounds__(256) void k_vp8_lf_sse(h264::Geometry g, const Vp8States* __restrict__ st,
                                                     const uint8_t* __restrict__ src_y,
                                                     const uint8_t* __restrict__ src_uv,
                                                     unsigned long long* __restrict__ sse_rows) {
    __shared__ uint32_t part[3][4];
    const Vp8FrameState& F = st->v;
    const int mby = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t e[3] = {0, 0, 0};
    // luma: 16 rows x coded_w, 4 samples per step; chroma: 8 rows x coded_w interleaved
    const int lw4 = g.coded_w / 4;
    for (int i = tid; i < 16 * lw4; i += 256) {
        const int r = i / lw4, x = (i % lw4) * 4, y = mby * 16 + r;
        if (y >= g.height) continue;
        const uint32_t a = *reinterpret_cast<const uint32_t*>(F.rec_y + (size_t)y * g.pitch + x);
        const uint32_t b = *reinterpret_cast<const uint32_t*>(src_y + (size_t)y * g.pitch + x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (int)((a >> (8 * k)) & 0xff) - (int)((b >> (8 * k)) & 0xff);
            e[0] += x + k < g.width ? (uint32_t)(d * d) : 0u;
        }
    }
    for (int i = tid; i < 8 * lw4; i += 256) {
        const int r = i / lw4, x = (i % lw4) * 4, cy = mby * 8 + r;
        if (2 * cy >= g.height) continue;
        const uint32_t a = *reinterpret_cast<const uint32_t*>(F.rec_uv + (size_t)cy * g.pitch + x);
        const uint32_t b = *reinterpret_cast<const uint32_t*>(src_uv + (size_t)cy * g.pitch + x);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (int)((a >> (8 * k)) & 0xff) - (int)((b >> (8 * k)) & 0xff);
            e[1 + (k & 1)] += 2 * ((x + k) >> 1) < g.width ? (uint32_t)(d * d) : 0u;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t w = (uint32_t)wsum((int)e[c]);
        if (lane == 0) part[c][wave] = w;
    }
    __syncthreads();
    if (tid < 3)
        sse_rows[3 * mby + tid] = (unsigned long long)part[tid][0] + part[tid][1] + part[tid][2] + part[tid][3];
}

// ------------------------------------------------------------------ hand-off to the host writer
// One workgroup per macroblock row: the rank of each coded macroblock within its row (ballots),
// its 800 level bytes to the mapped host buffer at slot row * mb_w + rank, every record with its
// slot.  Only coded macroblocks cross the bus.
__global__ __launch_bounds__(256) void k_vp8_gather(h264::Geometry g, const Vp8Mb* __restrict__ mbs,
                                                     const int16_t* __restrict__ lv, Vp8Mb* __restrict__ mb_host,
                                                     int16_t* __restrict__ lv_host) {
    // The records of a macroblock row and the levels of its coded macroblocks go to mapped host
    // memory -- over the host link, so only the blocks with a non-zero level travel (16 levels
    // each, compacted per row in macroblock order; a record's slot is its first block's index).
    // The writer expands them (vp8_gpu.cpp).  Each wave owns two 64-macroblock chunks of the row.
    __shared__ int wave_blk[4];
    __shared__ uint16_t bmap[4][128 * 25];  // per wave: (macroblock column << 5 | block) of every block to copy
    const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = g.mb_w, base = row * n;
    int nb[2] = {0, 0}, ex[2] = {0, 0};  // this lane's macroblock: blocks to copy, their offset in the wave
    uint32_t nzm[2] = {0u, 0u};
    int tot = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int i = wave * 128 + c * 64 + lane;
        nzm[c] = i < n ? (mbs[base + i].nz & 0x1FFFFFFu) : 0u;
        nb[c] = __popc(nzm[c]);
        int incl = nb[c];  // inclusive scan over the wave
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        ex[c] = tot + incl - nb[c];
        tot += __shfl(incl, 63, 64);
    }
    if (lane == 0) wave_blk[wave] = tot;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wave; ++w) off += wave_blk[w];
    const size_t row_blk = (size_t)base * kBlocks;  // the row's first block in lv_host
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int i = wave * 128 + c * 64 + lane;
        if (i < n) {
            Vp8Mb m = mbs[base + i];
            m.slot = (uint32_t)(row_blk + off + ex[c]);
            const uint4* srcw = reinterpret_cast<const uint4*>(&m);
            uint4* dst = reinterpret_cast<uint4*>(mb_host + base + i);
            dst[0] = srcw[0];
            dst[1] = srcw[1];
        }
        uint32_t z = nzm[c];
        for (int k = ex[c]; z; ++k) {
            const int bb = __builtin_ctz(z);
            z &= z - 1;
            bmap[wave][k] = (uint16_t)((i << 5) | bb);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // two uint4 per block, spread over the lanes: many copies in flight per wave
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(lv + (size_t)base * kCoefPerMb);
    uint4* __restrict__ dst = reinterpret_cast<uint4*>(lv_host + (row_blk + off) * 16);
#pragma unroll 4
    for (int t = lane; t < 2 * tot; t += 64) {
        const int e = bmap[wave][t >> 1];
        dst[t] = src[(size_t)(e >> 5) * (kCoefPerMb / 8) + (e & 31) * 2 + (t & 1)];
    }
}

}  // namespace

void launch_vp8_inter(const h264::Geometry& g, const Vp8DeviceBuffers& b, uint8_t* const hp_planes[4], int hp_pitch,
                      bool subpel, const uint8_t* src_y, const uint8_t* src_uv, hipStream_t stream, bool intra) {
    const int W = g.coded_w + 2 * h264::kHpelPad, H = g.coded_h + 2 * h264::kHpelPad;
    if (subpel)  // F (the same padded plane k_vp8_pad writes) plus the half-sample planes of the search
        h264::launch_hpel(g, b.me, hp_planes, hp_pitch, stream);
    else
        hipLaunchKernelGGL(k_vp8_pad, dim3((W / 4 + 255) / 256, H), dim3(256), 0, stream, g, b.st);
    h264::launch_me(g, b.me, src_y, stream);
    hipLaunchKernelGGL(k_vp8_inter, dim3(g.mb_w * g.mb_h), dim3(64), 0, stream, g, b.st, src_y, src_uv, b.me.mb, b.mb,
                       b.lv, b.ilist);
    if (intra) {
        hipLaunchKernelGGL(k_vp8_intra_cand, dim3((g.mb_w * g.mb_h + 3) / 4), dim3(256), 0, stream, g, b.st, src_y,
                           src_uv, b.mb, b.icand, b.ilist);
        hipLaunchKernelGGL(k_vp8_intra_code, dim3(kIntraCodeGrid), dim3(64), 0, stream, g, b.st, src_y, src_uv, b.mb,
                           b.lv, b.icand, b.ilist);
    }
}

void launch_vp8_key(const h264::Geometry& g, const Vp8DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                    hipStream_t stream, bool save_src, bool bpred) {
    if (save_src)  // the next inter frame's temporal classes compare against this source
        hipLaunchKernelGGL(k_vp8_save_src, dim3((g.coded_w / 4 + 255) / 256, g.coded_h), dim3(256), 0, stream, g, b.st,
                           src_y);
    if (bpred)  // the B_PRED plans, every macroblock at once, before the wavefront reads them
        hipLaunchKernelGGL(k_vp8_bpred_plan, dim3((g.mb_w * g.mb_h + 3) / 4), dim3(256), 0, stream, g, b.st, src_y, b.mb);
    hipLaunchKernelGGL(k_vp8_key, dim3(g.mb_h), dim3(64), 0, stream, g, b.st, src_y, src_uv, b.mb, b.lv,
                       b.line, b.err);
}

void launch_vp8_lf(const h264::Geometry& g, const Vp8DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                   hipStream_t stream) {
    hipLaunchKernelGGL(k_vp8_lf<kLfRows>, dim3((g.mb_h + kLfRows - 1) / kLfRows), dim3(64 * kLfRows), 0, stream, g, b.st,
                       b.mb, b.lf_line, b.err);
    hipLaunchKernelGGL(k_vp8_lf_sse, dim3(g.mb_h), dim3(256), 0, stream, g, b.st, src_y, src_uv, b.lf_sse);
}

void launch_vp8_gather(const h264::Geometry& g, const Vp8DeviceBuffers& b, hipStream_t stream) {
    hipLaunchKernelGGL(k_vp8_gather, dim3(g.mb_h), dim3(256), 0, stream, g, b.mb, b.lv, b.mb_host, b.lv_host);
}

}  // namespace vp8
}  // namespace mx
