// HIP/CDNA4 kernels of the H.264 encoder.
//
// Decomposition (gfx950: 256 CUs, wave64):
//  * k_me_full      one 256-thread workgroup per macroblock; the search window is staged
//                   in LDS and every lane scores (2R+1)^2/256 integer candidates with
//                   v_sad_u8 on byte-aligned dwords (v_alignbyte), then optional
//                   quarter-pel refinement; block-wide argmin via shuffles + LDS.
//  * k_inter_encode one wave per macroblock (4 per workgroup): motion compensation
//                   (6-tap qpel / bilinear chroma), 4x4 integer transform, quantisation,
//                   reconstruction into the reference frame.  Fully parallel over MBs.
//  * k_intra_analyze one wave per MB: open-loop Intra4x4 / Intra16x16 / chroma mode costs
//                   (SATD vs source-neighbour predictions) and the intra / inter decision.
//  * k_intra_wave   one workgroup per MB row (luma wave + chroma wave): closed-loop coding
//                   of the intra MBs in a diagonal wavefront with per-row progress flags.
//  * k_cavlc        one wave per macroblock: lane 0 codes the MB header (P_Skip decision,
//                   median mv prediction, cbp), lanes 1..27 code one residual block each;
//                   a wave prefix-sum places every lane's bits in an LDS slot.
//  * k_scan         one workgroup: skip runs, per-MB and per-slice bit offsets.
//  * k_pack         one thread per output word gathers the overlapping header / MB /
//                   trailer bits and stores the word straight into pinned host memory.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "../common/hip_check.h"
#include "h264_core.h"
#include "h264_deblock.h"
#include "h264_gpu.h"
#include "h264_mb.h"

namespace mx {
namespace h264 {

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// Bit writer that ORs 32-bit chunks into a zero-initialised word array starting at an
// arbitrary bit offset (atomicOr: neighbouring writers share boundary words).
template <bool kSwap>
struct OrWriter {
    uint32_t* dst;
    uint32_t pos;  // absolute bit position of the next chunk
    uint64_t acc;
    int nacc;
    uint32_t bits;

    __device__ __forceinline__ void init(uint32_t* d, uint32_t bitpos) {
        dst = d;
        pos = bitpos;
        acc = 0;
        nacc = 0;
        bits = 0;
    }
    __device__ __forceinline__ void emit(uint32_t w, int n) {  // w: n valid bits left-aligned
        const uint32_t wi = pos >> 5, sh = pos & 31;
        uint32_t a = w >> sh;
        if (a) atomicOr(dst + wi, kSwap ? bswap32(a) : a);
        if (sh && n > (int)(32 - sh)) {
            uint32_t b2 = w << (32 - sh);
            if (b2) atomicOr(dst + wi + 1, kSwap ? bswap32(b2) : b2);
        }
        pos += n;
    }
    __device__ __forceinline__ void put(uint32_t v, int n) {
        if (n <= 0) return;
        uint64_t m = (n == 32) ? 0xffffffffull : ((1ull << n) - 1);
        acc = (acc << n) | (v & m);
        nacc += n;
        bits += n;
        if (nacc >= 32) {
            emit((uint32_t)(acc >> (nacc - 32)), 32);
            nacc -= 32;
        }
    }
    __device__ __forceinline__ void flush() {
        if (nacc > 0) {
            emit((uint32_t)(acc << (32 - nacc)), nacc);
            nacc = 0;
            acc = 0;
        }
    }
};

// Sum of the four rows of 16 lanes, every lane gets it (whole wave active): v_permlane16_swap
// and v_permlane32_swap with both operands = v leave {v, v ^ 16} (then {v, v ^ 32}) on every
// lane, so the pair sum is the xor-16 / xor-32 butterfly step without a ds_bpermute round trip.
__device__ __forceinline__ uint32_t rows_sum(uint32_t v) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = r16[0] + r16[1];
    const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r32[0] + r32[1];
}
// Wave sum, every lane gets it (whole wave active): quad and row-of-16 sums with DPP
// (quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, row_ror 8), then rows_sum.
__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
    return (int)rows_sum((uint32_t)v);
}

// ------------------------------------------------------------------ half-pel planes
struct Planes {
    const uint8_t *f, *h, *v, *j;
    int pitch;
};
__device__ __forceinline__ Planes planes_of(const FrameState* fs) {
    return Planes{fs->hp_f, fs->hp_h, fs->hp_v, fs->hp_j, fs->hp_pitch};
}
// the motion search's planes (FrameState::me_*: the reference's unfiltered reconstruction)
__device__ __forceinline__ Planes me_planes_of(const FrameState* fs) {
    return fs->me_f ? Planes{fs->me_f, fs->me_h, fs->me_v, fs->me_j, fs->hp_pitch} : planes_of(fs);
}
// Quarter-sample luma value from the precomputed planes (Table 8-12); identical to
// luma_qpel() on the clamped reference.
__device__ __forceinline__ int qpel_planes(const Planes& P, int x4, int y4) {
    const int xi = x4 >> 2, yi = y4 >> 2, xf = x4 & 3, yf = y4 & 3;
    const int o = yi * P.pitch + xi;
    const int G = P.f[o];
    if ((xf | yf) == 0) return G;
    if (yf == 0) {
        const int b = P.h[o];
        if (xf == 2) return b;
        return ((xf == 1 ? G : (int)P.f[o + 1]) + b + 1) >> 1;
    }
    if (xf == 0) {
        const int hh = P.v[o];
        if (yf == 2) return hh;
        return ((yf == 1 ? G : (int)P.f[o + P.pitch]) + hh + 1) >> 1;
    }
    if (xf == 2 && yf == 2) return P.j[o];
    if (xf == 2) return ((yf == 1 ? (int)P.h[o] : (int)P.h[o + P.pitch]) + P.j[o] + 1) >> 1;
    if (yf == 2) return ((xf == 1 ? (int)P.v[o] : (int)P.v[o + 1]) + P.j[o] + 1) >> 1;
    const int bb = (yf == 1) ? P.h[o] : P.h[o + P.pitch];
    const int hh = (xf == 1) ? P.v[o] : P.v[o + 1];
    return (bb + hh + 1) >> 1;
}

// LDS-tiled F/H/V/J plane builder, 128x16 output tile per 256-thread workgroup.
//  1. the (16+5)-row clamped sample footprint is staged as whole dwords (aligned start
//     4 samples left of the tile; interior tiles use dword loads, border tiles clamp);
//  2. the horizontal 6-tap intermediates b1 for all 21 rows, 4 columns per item;
//  3. each lane produces a 4-pixel x 2-row block of all four planes from 7 sample dwords
//     and 7 b1 quads it shares between the two rows, and stores dwords (64 lanes = 2 rows
//     x 128 contiguous bytes per plane).
// The byte-per-lane version (64x16 tile) ran 19.6 us at 1080p (profiles/r01_final_check).
constexpr int kHpTW = 128, kHpTH = 16;
constexpr int kHpSW = kHpTW + 8;  // staged samples per row: padded x in [px0-4, px0+kHpTW+4)
__device__ __forceinline__ int byte_of(uint32_t w, int k) { return (int)((w >> (8 * k)) & 0xff); }
// Low bytes of a..d -> one dword via v_perm_b32.  Written as `clip255(v) << 8*j` ORs, the
// build produced 0xff in bytes 2-3 whenever sample 1 clamped from below to 0 (seen on the
// MI355X in test_hpel_planes_match_reference; a codegen issue, most likely in the narrowed
// clamp); v_perm reads only byte 0 of each operand, so stale high bits cannot leak.
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)d, (uint32_t)c, 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}
// Frame-state publication: the first kernel of a frame receives the state by value (kernel
// arguments, no extra dispatch) and stores it for the later kernels, replacing a per-frame
// 4.4 us host->device copy node (profiles/r02_b).  Under hipGraph capture the state still
// comes from a captured memcpy node (the captured argument would be stale), so `publish` = 0
// and the kernel reads the device copy.
struct StateArg {
    FrameState v;
    FrameState* dst;
    int publish;
    uint64_t* t_start;  // OutHeader::t_start of the frame (device), or nullptr
};
__device__ __forceinline__ void publish_state(const StateArg& a) {
    static_assert(sizeof(FrameState) % 4 == 0, "FrameState is copied as dwords");
    if (a.t_start && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.t_start = wall_clock64();
    if (a.publish && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < sizeof(FrameState) / 4)
        reinterpret_cast<uint32_t*>(a.dst)[threadIdx.x] = reinterpret_cast<const uint32_t*>(&a.v)[threadIdx.x];
}
__device__ __forceinline__ const FrameState& state_of(const StateArg& a) { return a.publish ? a.v : *a.dst; }

__global__ __launch_bounds__(256) void k_hpel(Geometry g, StateArg sa, uint8_t* __restrict__ pf,
                                              uint8_t* __restrict__ ph, uint8_t* __restrict__ pv,
                                              uint8_t* __restrict__ pj, int hp_pitch,
                                              const uint8_t* __restrict__ src) {
    __shared__ uint32_t smp[kHpTH + 5][kHpSW / 4];
    __shared__ int4 b1[kHpTH + 5][kHpTW / 4];  // 4 columns per entry
    publish_state(sa);
    const uint8_t* __restrict__ ref = src ? src : state_of(sa).ref_y;  // src: an explicit picture
    const int px0 = blockIdx.x * kHpTW, py0 = blockIdx.y * kHpTH;  // padded-plane coordinates
    const int W = g.coded_w + 2 * kHpelPad, H = g.coded_h + 2 * kHpelPad;
    const int tid = threadIdx.x;
    // smp[r][k] = picture sample (px0 - 4 + k - pad, py0 - 2 + r - pad), clamped to the picture
    const int xs = px0 - 4 - kHpelPad, ys = py0 - 2 - kHpelPad;
    const bool interior = xs >= 0 && xs + kHpSW <= g.coded_w && ys >= 0 && ys + kHpTH + 5 <= g.coded_h &&
                          (g.pitch & 3) == 0 && (reinterpret_cast<uintptr_t>(ref) & 3) == 0;
    for (int i = tid; i < (kHpTH + 5) * (kHpSW / 4); i += 256) {
        const int r = i / (kHpSW / 4), k4 = i - r * (kHpSW / 4);
        uint32_t w;
        if (interior) {
            w = *reinterpret_cast<const uint32_t*>(ref + (size_t)(ys + r) * g.pitch + xs + 4 * k4);
        } else {
            w = 0;
            for (int k = 0; k < 4; ++k)
                w |= (uint32_t)ref_px(ref, g.pitch, g.coded_w, g.coded_h, xs + 4 * k4 + k, ys + r) << (8 * k);
        }
        smp[r][k4] = w;
    }
    __syncthreads();
    // b1 at output column c uses samples k = c+2 .. c+7; a 4-column group c = 4q needs
    // staged dwords q, q+1, q+2
    for (int i = tid; i < (kHpTH + 5) * (kHpTW / 4); i += 256) {
        const int r = i / (kHpTW / 4), q = i - r * (kHpTW / 4);
        const uint32_t w0 = smp[r][q], w1 = smp[r][q + 1], w2 = smp[r][q + 2];
        int s[12];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[k] = byte_of(w0, k);
            s[4 + k] = byte_of(w1, k);
            s[8 + k] = byte_of(w2, k);
        }
        int t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = tap6(s[j + 2], s[j + 3], s[j + 4], s[j + 5], s[j + 6], s[j + 7]);
        b1[r][q] = make_int4(t[0], t[1], t[2], t[3]);
    }
    __syncthreads();
    const int q = tid & (kHpTW / 4 - 1), r0 = (tid / (kHpTW / 4)) * 2;  // 32 groups x 8 row pairs
    const int x = px0 + 4 * q;
    if (x >= W) return;  // W % 4 == 0: a group is wholly inside or outside
    // output row r reads staged rows r .. r+5 (centre r+2); the pair shares rows r0+1 .. r0+5
    int sv[7][4], bv[7][4];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint32_t w = smp[r0 + k][q + 1];  // samples k = 4q+4 .. 4q+7 = output columns 4q .. 4q+3
        const int4 bb = b1[r0 + k][q];
#pragma unroll
        for (int j = 0; j < 4; ++j) sv[k][j] = byte_of(w, j);
        bv[k][0] = bb.x;
        bv[k][1] = bb.y;
        bv[k][2] = bb.z;
        bv[k][3] = bb.w;
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int y = py0 + r0 + rr;
        if (y >= H) break;
        int Hs[4], Vs[4], Js[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            Hs[j] = clip255((bv[rr + 2][j] + 16) >> 5);  // centre row of this output row: rr + 2
            const int v1 = tap6(sv[rr][j], sv[rr + 1][j], sv[rr + 2][j], sv[rr + 3][j], sv[rr + 4][j], sv[rr + 5][j]);
            Vs[j] = clip255((v1 + 16) >> 5);
            const int j1 = tap6(bv[rr][j], bv[rr + 1][j], bv[rr + 2][j], bv[rr + 3][j], bv[rr + 4][j], bv[rr + 5][j]);
            Js[j] = clip255((j1 + 512) >> 10);
        }
        const size_t o = (size_t)y * hp_pitch + x;
        *reinterpret_cast<uint32_t*>(pf + o) = smp[r0 + rr + 2][q + 1];
        *reinterpret_cast<uint32_t*>(ph + o) = pack4(Hs[0], Hs[1], Hs[2], Hs[3]);
        *reinterpret_cast<uint32_t*>(pv + o) = pack4(Vs[0], Vs[1], Vs[2], Vs[3]);
        *reinterpret_cast<uint32_t*>(pj + o) = pack4(Js[0], Js[1], Js[2], Js[3]);
    }
}

// Quarter-sample luma value from an LDS-staged 18x18 footprint of the four planes
// (sp[0] F, sp[1] H, sp[2] V, sp[3] J; local origin one sample up-left of the integer
// match); exactly qpel_planes() on the same samples.
constexpr int kSpW = 20;
__device__ __forceinline__ int qpel_lds(const uint8_t (*sp)[18][kSpW], int x4, int y4) {
    const int xi = x4 >> 2, yi = y4 >> 2, xf = x4 & 3, yf = y4 & 3;
    const int G = sp[0][yi][xi];
    if ((xf | yf) == 0) return G;
    if (yf == 0) {
        const int b = sp[1][yi][xi];
        if (xf == 2) return b;
        return ((xf == 1 ? G : (int)sp[0][yi][xi + 1]) + b + 1) >> 1;
    }
    if (xf == 0) {
        const int hh = sp[2][yi][xi];
        if (yf == 2) return hh;
        return ((yf == 1 ? G : (int)sp[0][yi + 1][xi]) + hh + 1) >> 1;
    }
    if (xf == 2 && yf == 2) return sp[3][yi][xi];
    if (xf == 2) return ((yf == 1 ? (int)sp[1][yi][xi] : (int)sp[1][yi + 1][xi]) + sp[3][yi][xi] + 1) >> 1;
    if (yf == 2) return ((xf == 1 ? (int)sp[2][yi][xi] : (int)sp[2][yi][xi + 1]) + sp[3][yi][xi] + 1) >> 1;
    const int bb = (yf == 1) ? sp[1][yi][xi] : sp[1][yi + 1][xi];
    const int hh = (xf == 1) ? sp[2][yi][xi] : sp[2][yi][xi + 1];
    return (bb + hh + 1) >> 1;
}

// ------------------------------------------------------------------ motion estimation
constexpr int kMaxRange = 32;
static_assert(kMaxRange + 2 <= kHpelPad, "search window must stay inside the padded planes");
constexpr int kWinStride = 16 + 2 * kMaxRange + 8;  // bytes per LDS window row (dword padded)

// Four waves.  (Five -- the +-16 search's 297 candidate tasks in one pass of 320 threads instead
// of 1.16 passes of 256 -- measured slower: 45 -> 54 us at 1080p, 78 -> 110 us at 4K, the larger
// workgroups costing more in occupancy than the shorter second pass saved: profiles/r04_h264.)
constexpr int kMeThreads = 256, kMeWaves = kMeThreads / 64;
__device__ __forceinline__ void me_full_body(const Geometry& g, const FrameState* __restrict__ fs,
                                             const uint8_t* __restrict__ src_y, MbInfo* __restrict__ mbs) {
    __shared__ uint32_t win32[(16 + 2 * kMaxRange) * kWinStride / 4];
    __shared__ uint32_t srcw[64];
    __shared__ unsigned long long red[kMeWaves];
    __shared__ uint32_t cand_cost[8];
    __shared__ uint32_t s_sad0[4];

    const int mbi = blockIdx.x;  // default dispatch order (XCD mappings measured: profiles/r01_xcd)
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    const int x0 = mbx * 16, y0 = mby * 16;
    const int tid = threadIdx.x, lane = tid & 63;
    const int R = me_range(fs->search_range);
    const int W = 16 + 2 * R;
    const Planes P = me_planes_of(fs);  // the unfiltered reference when it was deblocked
    const int lambda = lambda_sad(fs->qp);

    // static-block early exit first: SAD of the zero vector from one source and one reference
    // pixel per thread (same rule as the CPU encoder), so the ~70 % static MBs of a desktop
    // never load the search window (a separate static pre-pass kernel feeding a list of the
    // moving MBs was measured slower: its atomic list append serialises, profiles/r02_me)
    constexpr int kWs4 = kWinStride / 4;
    {
        if (tid < 64) {  // one wave: a dword of source and reference per lane, v_sad_u8
            const int r = tid >> 2, c4 = (tid & 3) * 4;
            const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c4);
            const uint32_t rw = *reinterpret_cast<const uint32_t*>(P.f + (y0 + r) * P.pitch + x0 + c4);
            const int d = wave_sum((int)__builtin_amdgcn_sad_u8(sw, rw, 0u));
            if (tid == 0) s_sad0[0] = (uint32_t)d;
        }
        __syncthreads();
        const uint32_t sad0 = s_sad0[0];
        if (sad0 <= static_sad(fs->qp)) {
            if (tid == 0) {
                MbInfo& m = mbs[mbi];
                m.mvx = 0;
                m.mvy = 0;
                m.part = kPart16x16;
                m.pmv[0] = m.pmv[1] = m.pmv[2] = m.pmv[3] = 0;
            }
            return;  // uniform across the workgroup
        }
    }
    // search window from the padded full-sample plane with dword loads (x0 - R is a
    // multiple of 4 and R + 2 <= kHpelPad: no clamping, no byte gathers)
    const bool t256 = tid < 256;  // the threads of the 256-thread refinement layouts
    for (int i = tid; i < W * kWs4; i += kMeThreads) {
        const int wy = i / kWs4, wx4 = (i - wy * kWs4) * 4;
        win32[i] = (wx4 < W) ? *reinterpret_cast<const uint32_t*>(P.f + (y0 - R + wy) * P.pitch + (x0 - R + wx4)) : 0u;
    }
    if (tid < 64) {
        const int r = tid >> 2, c = (tid & 3) * 4;
        srcw[tid] = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c);
    }
    __syncthreads();

    // Each thread scores four horizontally adjacent candidates per step: their 16x16 blocks
    // share one dword-aligned 20-byte row span of the window, so every row costs 5 LDS reads
    // (instead of 5 per candidate), 12 v_alignbyte and 16 v_sad_u8.
    const int side = 2 * R + 1, gw = (side + 3) >> 2, ngroups = side * gw;
    unsigned long long best = ~0ull;
    const bool coarse = fs->me_coarse != 0;
    // coarse mode (me_coarse): the even-offset grid first -- two candidates per thread (window
    // shifts 0 and 2 of a dword group), (R + 1) * gw tasks in one pass -- then the 8 integer
    // neighbours of its best (me_search_cpu does the same)
    const bool parts = fs->partitions != 0;  // 16x8 / 8x16 partitionings searched too (me_search_parts_cpu)
    const int ntask = (coarse && !parts) ? (R + 1) * gw : 0;
    auto mkey = [&](uint32_t sad, int dxr, int dyr) {
        const int dx = dxr - R, dy = dyr - R;
        const uint32_t cost = me_cost(sad, lambda, 4 * dx, 4 * dy);
        const uint32_t dist = (uint32_t)(abs(dx) + abs(dy));
        return ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)(dyr * side + dxr);
    };
    // partitions: per candidate the SAD of each 8x8 quadrant (TL, TR, BL, BR); the 16x16 key is
    // their sum (so the 16x16 decision is unchanged) and shapes T / B / L / R keep their own best
    unsigned long long pb[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    auto kmin = [](unsigned long long a, unsigned long long c) { return c < a ? c : a; };
    auto visit_quads = [&](const uint32_t* qd, int dxr, int dyr) {
        best = kmin(best, mkey(qd[0] + qd[1] + qd[2] + qd[3], dxr, dyr));
        pb[0] = kmin(pb[0], mkey(qd[0] + qd[1], dxr, dyr));
        pb[1] = kmin(pb[1], mkey(qd[2] + qd[3], dxr, dyr));
        pb[2] = kmin(pb[2], mkey(qd[0] + qd[2], dxr, dyr));
        pb[3] = kmin(pb[3], mkey(qd[1] + qd[3], dxr, dyr));
    };
    if (parts) {
        // tasks: the even grid (coarse, shifts 0 and 2 of a dword group) or every group (shifts 0..3)
        const int nsh = coarse ? 2 : 4, ntp = coarse ? (R + 1) * gw : ngroups;
        for (int q = tid; q < ntp; q += kMeThreads) {
            const int dyr = coarse ? 2 * (q / gw) : q / gw, g = q % gw;
            uint32_t acc[4][4];  // [shift index][quadrant]
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0;
#pragma unroll 2
            for (int r = 0; r < 16; ++r) {
                const int a = (dyr + r) * kWs4 + g, hq = r < 8 ? 0 : 2;
                const uint32_t w0 = win32[a], w1 = win32[a + 1], w2 = win32[a + 2], w3 = win32[a + 3], w4 = win32[a + 4];
                const uint32_t s0 = srcw[r * 4 + 0], s1 = srcw[r * 4 + 1], s2 = srcw[r * 4 + 2], s3 = srcw[r * 4 + 3];
#pragma unroll
                for (int si = 0; si < 4; ++si) {
                    if (si >= nsh) break;
                    const int sh = coarse ? 2 * si : si;
                    const uint32_t a0 = sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
                    const uint32_t a1 = sh ? __builtin_amdgcn_alignbyte(w2, w1, sh) : w1;
                    const uint32_t a2 = sh ? __builtin_amdgcn_alignbyte(w3, w2, sh) : w2;
                    const uint32_t a3 = sh ? __builtin_amdgcn_alignbyte(w4, w3, sh) : w3;
                    uint32_t lft = hq ? acc[si][2] : acc[si][0], rgt = hq ? acc[si][3] : acc[si][1];
                    lft = __builtin_amdgcn_sad_u8(a1, s1, __builtin_amdgcn_sad_u8(a0, s0, lft));
                    rgt = __builtin_amdgcn_sad_u8(a3, s3, __builtin_amdgcn_sad_u8(a2, s2, rgt));
                    if (hq) {
                        acc[si][2] = lft;
                        acc[si][3] = rgt;
                    } else {
                        acc[si][0] = lft;
                        acc[si][1] = rgt;
                    }
                }
            }
#pragma unroll
            for (int si = 0; si < 4; ++si) {
                if (si >= nsh) break;
                const int dxr = 4 * g + (coarse ? 2 * si : si);
                if (dxr >= side) break;
                visit_quads(acc[si], dxr, dyr);
            }
        }
    }
    for (int q = tid; q < ntask; q += kMeThreads) {
        const int dyr = 2 * (q / gw), g = q % gw;
        uint32_t s0a = 0, s2a = 0;
#pragma unroll 4
        for (int r = 0; r < 16; ++r) {
            const int a = (dyr + r) * kWs4 + g;
            const uint32_t w0 = win32[a], w1 = win32[a + 1], w2 = win32[a + 2], w3 = win32[a + 3], w4 = win32[a + 4];
            const uint32_t s0 = srcw[r * 4 + 0], s1 = srcw[r * 4 + 1], s2 = srcw[r * 4 + 2], s3 = srcw[r * 4 + 3];
            s0a = __builtin_amdgcn_sad_u8(w0, s0, s0a);
            s0a = __builtin_amdgcn_sad_u8(w1, s1, s0a);
            s0a = __builtin_amdgcn_sad_u8(w2, s2, s0a);
            s0a = __builtin_amdgcn_sad_u8(w3, s3, s0a);
            s2a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, 2), s0, s2a);
            s2a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w2, w1, 2), s1, s2a);
            s2a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w3, w2, 2), s2, s2a);
            s2a = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w4, w3, 2), s3, s2a);
        }
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int dxr = 4 * g + 2 * h2;
            if (dxr >= side) break;
            const int dx = dxr - R, dy = dyr - R, c = dyr * side + dxr;
            const uint32_t cost = me_cost(h2 ? s2a : s0a, lambda, 4 * dx, 4 * dy);
            const uint32_t dist = (uint32_t)(abs(dx) + abs(dy));
            const unsigned long long key = ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)c;
            best = key < best ? key : best;
        }
    }
    for (int q = tid; q < ((coarse || parts) ? 0 : ngroups); q += kMeThreads) {
        const int dyr = q / gw, g = q - dyr * gw;
        uint32_t sad[4] = {0, 0, 0, 0};
#pragma unroll 2
        for (int r = 0; r < 16; ++r) {
            const int a = (dyr + r) * kWs4 + g;
            const uint32_t w0 = win32[a], w1 = win32[a + 1], w2 = win32[a + 2], w3 = win32[a + 3], w4 = win32[a + 4];
            const uint32_t s0 = srcw[r * 4 + 0], s1 = srcw[r * 4 + 1], s2 = srcw[r * 4 + 2], s3 = srcw[r * 4 + 3];
            sad[0] = __builtin_amdgcn_sad_u8(w0, s0, sad[0]);
            sad[0] = __builtin_amdgcn_sad_u8(w1, s1, sad[0]);
            sad[0] = __builtin_amdgcn_sad_u8(w2, s2, sad[0]);
            sad[0] = __builtin_amdgcn_sad_u8(w3, s3, sad[0]);
#pragma unroll
            for (int sh = 1; sh < 4; ++sh) {
                uint32_t t = sad[sh];
                t = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, sh), s0, t);
                t = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w2, w1, sh), s1, t);
                t = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w3, w2, sh), s2, t);
                t = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w4, w3, sh), s3, t);
                sad[sh] = t;
            }
        }
#pragma unroll
        for (int sh = 0; sh < 4; ++sh) {
            const int dxr = 4 * g + sh;
            if (dxr >= side) break;
            const int dx = dxr - R, dy = dyr - R, c = dyr * side + dxr;
            const uint32_t cost = me_cost(sad[sh], lambda, 4 * dx, 4 * dy);
            const uint32_t dist = (uint32_t)(abs(dx) + abs(dy));
            const unsigned long long key = ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)c;
            best = key < best ? key : best;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long other = __shfl_xor(best, o, 64);
        best = other < best ? other : best;
    }
    if (lane == 0) red[tid >> 6] = best;
    __shared__ unsigned long long pred4[4][kMeWaves];  // partitions: [shape][wave]
    if (parts) {
#pragma unroll
        for (int sh = 0; sh < 4; ++sh) {
            unsigned long long v = pb[sh];
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long other = __shfl_xor(v, o, 64);
                v = other < v ? other : v;
            }
            if (lane == 0) pred4[sh][tid >> 6] = v;
        }
    }
    __syncthreads();
    unsigned long long b = red[0];
    for (int i = 1; i < kMeWaves; ++i) b = red[i] < b ? red[i] : b;
    unsigned long long pbest[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    if (parts)
        for (int sh = 0; sh < 4; ++sh)
            for (int i = 0; i < kMeWaves; ++i) pbest[sh] = pred4[sh][i] < pbest[sh] ? pred4[sh][i] : pbest[sh];
    if (parts && coarse) {
        // the 8 integer neighbours of each partition's grid best: 32 (shape, neighbour) pairs of
        // 128-sample rectangles, 8 lanes (16 samples) each
        __shared__ unsigned long long pnkey[4][8];
        const int ev = (tid & 255) >> 3, sub = tid & 7, sh = ev >> 3, k = ev & 7;
        const int cb0 = (int)(pbest[sh] & 0xffff), bxr = cb0 % side, byr = cb0 / side;
        int ddx, ddy;
        subpel_offset(k, &ddx, &ddy);
        const int nxr = bxr + ddx, nyr = byr + ddy;
        const bool inside = t256 && nxr >= 0 && nxr < side && nyr >= 0 && nyr < side;  // uniform per 8-lane group
        int d = 0;
        if (inside) {
            // T / B: one 16-sample row each (row sub of the half); L / R: two 8-sample rows
            const uint8_t* wb = reinterpret_cast<const uint8_t*>(win32);
            const uint8_t* sb = reinterpret_cast<const uint8_t*>(srcw);
            for (int part_row = 0; part_row < 2; ++part_row) {
                const int rr = sh < 2 ? (sh == 0 ? sub : 8 + sub) : 2 * sub + part_row;
                const int c0 = sh < 2 ? 8 * part_row : (sh == 2 ? 0 : 8);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    d += abs((int)sb[rr * 16 + c0 + j] - (int)wb[(nyr + rr) * kWinStride + nxr + c0 + j]);
            }
        }
        for (int o = 4; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        if (t256 && sub == 0) pnkey[sh][k] = inside ? mkey((uint32_t)d, nxr, nyr) : ~0ull;
        __syncthreads();
        for (int s2 = 0; s2 < 4; ++s2)
            for (int i = 0; i < 8; ++i) pbest[s2] = pnkey[s2][i] < pbest[s2] ? pnkey[s2][i] : pbest[s2];
    }
    if (coarse) {  // the 8 integer neighbours of the grid best: one per 32-lane group
        __shared__ unsigned long long nkey[8];
        const int cb0 = (int)(b & 0xffff), bxr = cb0 % side, byr = cb0 / side;
        const int k = (tid & 255) >> 5, sub = tid & 31, py = sub >> 1, px0 = (sub & 1) * 8;
        int ddx, ddy;
        subpel_offset(k, &ddx, &ddy);
        const int nxr = bxr + ddx, nyr = byr + ddy;
        const bool inside = t256 && nxr >= 0 && nxr < side && nyr >= 0 && nyr < side;  // uniform per group
        int d = 0;
        if (inside) {
            const uint8_t* wrow = reinterpret_cast<const uint8_t*>(win32) + (nyr + py) * kWinStride + nxr + px0;
            const uint32_t s0 = srcw[py * 4 + (px0 >> 2)], s1 = srcw[py * 4 + (px0 >> 2) + 1];
#pragma unroll
            for (int j = 0; j < 8; ++j) d += abs((int)(((j < 4 ? s0 : s1) >> (8 * (j & 3))) & 0xff) - (int)wrow[j]);
        }
        for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        if (t256 && sub == 0) {
            const int dx = nxr - R, dy = nyr - R;
            const uint32_t cost = me_cost((uint32_t)d, lambda, 4 * dx, 4 * dy);
            const uint32_t dist = (uint32_t)(abs(dx) + abs(dy));
            nkey[k] = inside ? (((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)(nyr * side + nxr)) : ~0ull;
        }
        __syncthreads();
        for (int i = 0; i < 8; ++i) b = nkey[i] < b ? nkey[i] : b;
    }
    const int cbest = (int)(b & 0xffff);
    int mvx = 4 * ((cbest % side) - R), mvy = 4 * ((cbest / side) - R);

    if (parts) {
        // shape decision on the integer costs: 16x16 unless a partitioning's two costs + 2 lambda
        // (mb_type bits) are lower, 16x8 before 8x16 on ties
        const uint32_t c16 = (uint32_t)(b >> 32);
        const uint32_t chz = (uint32_t)(pbest[0] >> 32) + (uint32_t)(pbest[1] >> 32) + 2u * (uint32_t)lambda;
        const uint32_t cvt = (uint32_t)(pbest[2] >> 32) + (uint32_t)(pbest[3] >> 32) + 2u * (uint32_t)lambda;
        const int part = (c16 <= chz && c16 <= cvt) ? kPart16x16 : (chz <= cvt ? kPart16x8 : kPart8x16);
        if (part != kPart16x16) {
            const int s0 = part == kPart16x8 ? 0 : 2;  // pbest index of partition 0
            int pvx[2], pvy[2];
            uint32_t pcost[2];
            for (int i = 0; i < 2; ++i) {
                const int cb = (int)(pbest[s0 + i] & 0xffff);
                pvx[i] = 4 * ((cb % side) - R);
                pvy[i] = 4 * ((cb / side) - R);
                pcost[i] = (uint32_t)(pbest[s0 + i] >> 32);
            }
            if (fs->subpel) {
                // half then quarter pel per partition over its own rectangle: an 18x18 footprint
                // per partition, 16 lanes (8 samples each) per candidate, both partitions at once
                __shared__ uint8_t psp[2][4][18][kSpW];
                __shared__ uint32_t pcand[2][8];
                for (int i = tid; i < 2 * 4 * 18 * 18; i += kMeThreads) {
                    const int pi = i / (4 * 324), rem0 = i - pi * 4 * 324;
                    const int pl = rem0 / 324, rem = rem0 - pl * 324, r = rem / 18, c = rem - r * 18;
                    const uint8_t* base = pl == 0 ? P.f : pl == 1 ? P.h : pl == 2 ? P.v : P.j;
                    const int ix = x0 + (pvx[pi] >> 2) - 1, iy = y0 + (pvy[pi] >> 2) - 1;
                    psp[pi][pl][r][c] = base[(iy + r) * P.pitch + ix + c];
                }
                __syncthreads();
                const int pi = (tid & 255) >> 7, k = (tid >> 4) & 7, sub = tid & 15;
                // the 8 samples of this lane inside the partition rectangle
                const int rx = part == kPart8x16 ? 8 * pi : 0, ry = part == kPart16x8 ? 8 * pi : 0;
                const int prow = part == kPart16x8 ? (sub >> 1) : sub, pcol = part == kPart16x8 ? (sub & 1) * 8 : 0;
                const int yy = ry + prow, xx = rx + pcol;
                const uint32_t s0w = srcw[yy * 4 + (xx >> 2)], s1w = srcw[yy * 4 + (xx >> 2) + 1];
                const int ivx = pvx[pi], ivy = pvy[pi];  // the integer match the footprint is staged around
                const int base_x4 = xx * 4 + 4 - ivx, base_y4 = yy * 4 + 4 - ivy;
                for (int step = 2; step >= 1; step >>= 1) {
                    int ddx, ddy;
                    subpel_offset(k, &ddx, &ddy);
                    const int cx = pvx[pi] + ddx * step, cy = pvy[pi] + ddy * step;
                    int d = 0;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int sv = (int)(((j < 4 ? s0w : s1w) >> (8 * (j & 3))) & 0xff);
                        d += abs(sv - qpel_lds(psp[pi], base_x4 + 4 * j + cx, base_y4 + cy));
                    }
                    for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
                    __syncthreads();  // the previous step's readers are done with pcand
                    if (t256 && sub == 0) pcand[pi][k] = me_cost((uint32_t)d, lambda, cx, cy);
                    __syncthreads();
                    for (int q = 0; q < 2; ++q) {
                        int bdx = 0, bdy = 0;
                        uint32_t bcost = pcost[q];
                        for (int kk = 0; kk < 8; ++kk) {
                            const uint32_t cc = pcand[q][kk];
                            if (cc < bcost) {
                                int ex, ey;
                                subpel_offset(kk, &ex, &ey);
                                bcost = cc;
                                bdx = ex * step;
                                bdy = ey * step;
                            }
                        }
                        pvx[q] += bdx;
                        pvy[q] += bdy;
                        pcost[q] = bcost;
                    }
                }
            }
            if (tid == 0) {
                MbInfo& m = mbs[mbi];
                m.mvx = (int16_t)mvx;  // the integer 16x16 vector (unused by the partitioned MB)
                m.mvy = (int16_t)mvy;
                m.part = (uint8_t)part;
                m.pmv[0] = (int16_t)pvx[0];
                m.pmv[1] = (int16_t)pvy[0];
                m.pmv[2] = (int16_t)pvx[1];
                m.pmv[3] = (int16_t)pvy[1];
            }
            return;  // uniform
        }
    }

    if (fs->subpel) {
        // half-pel then quarter-pel around the integer match.  Every candidate of both steps
        // lies in one 18x18 footprint of the F/H/V/J planes (the integer match +-1 sample),
        // staged into LDS once with independent byte loads; the 8 neighbours of a step are
        // scored at once, one per 32-lane half-wave group (8 pixels per lane, source from
        // srcw), a 5-step xor shuffle reduces each group, one barrier publishes the costs.
        __shared__ uint8_t sp[4][18][kSpW];
        const int ix = x0 + (mvx >> 2) - 1, iy = y0 + (mvy >> 2) - 1;
        for (int i = tid; i < 4 * 18 * 18; i += kMeThreads) {
            const int pl = i / 324, rem = i - pl * 324, r = rem / 18, c = rem - r * 18;
            const uint8_t* base = pl == 0 ? P.f : pl == 1 ? P.h : pl == 2 ? P.v : P.j;
            sp[pl][r][c] = base[(iy + r) * P.pitch + ix + c];
        }
        __syncthreads();
        uint32_t cur_cost = (uint32_t)(b >> 32);
        const int k = (tid & 255) >> 5, sub = tid & 31;
        const int py = sub >> 1, px0 = (sub & 1) * 8;
        const uint32_t s0 = srcw[py * 4 + (px0 >> 2)], s1 = srcw[py * 4 + (px0 >> 2) + 1];
        const int base_x4 = px0 * 4 + 4 - mvx, base_y4 = py * 4 + 4 - mvy;  // local qpel coords = base + candidate mv
        for (int step = 2; step >= 1; step >>= 1) {
            int ddx, ddy;
            subpel_offset(k, &ddx, &ddy);
            const int cx = mvx + ddx * step, cy = mvy + ddy * step;
            int d = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int sv = (int)(((j < 4 ? s0 : s1) >> (8 * (j & 3))) & 0xff);
                d += abs(sv - qpel_lds(sp, base_x4 + 4 * j + cx, base_y4 + cy));
            }
            for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
            __syncthreads();  // previous step's readers are done with cand_cost
            if (t256 && sub == 0) cand_cost[k] = me_cost((uint32_t)d, lambda, cx, cy);
            __syncthreads();
            int bdx = 0, bdy = 0;
            uint32_t bcost = cur_cost;
            for (int kk = 0; kk < 8; ++kk) {
                const uint32_t cc = cand_cost[kk];
                if (cc < bcost) {
                    int ex, ey;
                    subpel_offset(kk, &ex, &ey);
                    bcost = cc;
                    bdx = ex * step;
                    bdy = ey * step;
                }
            }
            mvx += bdx;
            mvy += bdy;
            cur_cost = bcost;
        }
    }
    if (tid == 0) {
        MbInfo& m = mbs[mbi];
        m.mvx = (int16_t)mvx;
        m.mvy = (int16_t)mvy;
        m.part = kPart16x16;
        m.pmv[0] = m.pmv[1] = m.pmv[2] = m.pmv[3] = 0;
    }
}

// The search reads the published frame state (the analysis stream's first kernel wrote it) or,
// on the side stream beside the previous picture's in-loop filter, a copy passed by value
// (a separate kernel, so the common launch keeps its small argument block)
__global__ __launch_bounds__(kMeThreads) void k_me_full(Geometry g, const FrameState* __restrict__ fs,
                                                  const uint8_t* __restrict__ src_y, MbInfo* __restrict__ mbs) {
    me_full_body(g, fs, src_y, mbs);
}
__global__ __launch_bounds__(kMeThreads) void k_me_full_val(Geometry g, FrameState fs,
                                                      const uint8_t* __restrict__ src_y, MbInfo* __restrict__ mbs) {
    me_full_body(g, &fs, src_y, mbs);
}

// ------------------------------------------------------------------ inter encode
// One MB per wave, 4x4 blocks in "row" layout: lane 4b + r holds row r of block b (luma: all
// 64 lanes = 16 blocks; chroma: lanes 0..31 = 8 blocks).  Both 1-D passes of every transform
// run in-lane on a row, the column pass gathers the block's four rows with DPP quad
// broadcasts (no LDS round trips); the integer arithmetic is exactly fdct4x4 / idct4x4 /
// hadamard4x4 / quant4x4 / dequant4x4 (rows first, then columns), so the bitstream is
// unchanged.  A block-per-lane layout left 40 of 64 lanes idle in the transform phase.
template <int K>
__device__ __forceinline__ int qbc(int v) {  // lane K of this lane's quad (quad_perm [K,K,K,K])
    return __builtin_amdgcn_mov_dpp(v, K * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ int quad_sum(int v) { return qbc<0>(v) + qbc<1>(v) + qbc<2>(v) + qbc<3>(v); }

// forward core transform of row r of a block whose rows sit in the quad: y = row r of Cf X Cf^T
__device__ __forceinline__ void fdct_row(const int* x, int r, int* y) {
    const int s03 = x[0] + x[3], d03 = x[0] - x[3], s12 = x[1] + x[2], d12 = x[1] - x[2];
    const int t[4] = {s03 + s12, 2 * d03 + d12, s03 - s12, d03 - 2 * d12};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int a0 = qbc<0>(t[c]), a1 = qbc<1>(t[c]), a2 = qbc<2>(t[c]), a3 = qbc<3>(t[c]);
        const int u03 = a0 + a3, e03 = a0 - a3, u12 = a1 + a2, e12 = a1 - a2;
        y[c] = r == 0 ? u03 + u12 : r == 1 ? 2 * e03 + e12 : r == 2 ? u03 - u12 : e03 - 2 * e12;
    }
}
// inverse core transform: residual row r from dequantised row d
__device__ __forceinline__ void idct_row(const int* d, int r, int* out) {
    const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
    const int f[4] = {e0 + e3, e1 + e2, e1 - e2, e0 - e3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int b0 = qbc<0>(f[c]), b1 = qbc<1>(f[c]), b2 = qbc<2>(f[c]), b3 = qbc<3>(f[c]);
        const int g0 = b0 + b2, g1 = b0 - b2, g2 = (b1 >> 1) - b3, g3 = b1 + (b3 >> 1);
        const int v = r == 0 ? g0 + g3 : r == 1 ? g1 + g2 : r == 2 ? g1 - g2 : g0 - g3;
        out[c] = (v + 32) >> 6;
    }
}
// sum |Hadamard coefficients| of row r (satd4x4 before its halving)
__device__ __forceinline__ int had_row_abs(const int* x, int r) {
    const int t[4] = {x[0] + x[1] + x[2] + x[3], x[0] + x[1] - x[2] - x[3], x[0] - x[1] - x[2] + x[3],
                      x[0] - x[1] + x[2] - x[3]};
    int s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int a = qbc<0>(t[c]), b = qbc<1>(t[c]), cc = qbc<2>(t[c]), d = qbc<3>(t[c]);
        const int v = r == 0 ? a + b + cc + d : r == 1 ? a + b - cc - d : r == 2 ? a - b - cc + d : a - b + cc - d;
        s += v < 0 ? -v : v;
    }
    return s;
}
// quant4x4 / dequant4x4 on row r (start = 1: the DC position is skipped)
__device__ __forceinline__ int quant_row(const int* y, int r, int qp, bool intra, int start, int* z) {
    const int qm = qp % 6, qbits = 15 + qp / 6;
    const int f = intra ? ((1 << qbits) / 3) : ((1 << qbits) / 6);
    int nz = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int i = r * 4 + c;
        if (i < start) {
            z[c] = 0;
            continue;
        }
        const int a = y[c] < 0 ? -y[c] : y[c];
        int q = (int)(((int64_t)a * kQuantMF[qm][kPosClass[i]] + f) >> qbits);
        q = q > kMaxLevel ? kMaxLevel : q;
        z[c] = y[c] < 0 ? -q : q;
        nz += (q != 0);
    }
    return nz;
}
__device__ __forceinline__ void dequant_row(const int* z, int r, int qp, int* d) {
    const int qm = qp % 6, qs = qp / 6;
#pragma unroll
    for (int c = 0; c < 4; ++c) d[c] = z[c] * kDequantV[qm][kPosClass[r * 4 + c]] * (1 << qs);
}

__global__ __launch_bounds__(256) void k_inter_encode(Geometry g, const FrameState* __restrict__ fs,
                                                       const uint8_t* __restrict__ src_y,
                                                       const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs,
                                                       int16_t* __restrict__ coef, uint32_t* __restrict__ mb_sse,
                                                       int* __restrict__ wave_prog) {
    __shared__ uint8_t pred[4][384];
    __shared__ int16_t res[4][384];
    __shared__ int cdc[4][8];
    __shared__ int cdc_nz[4][2];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nmb = g.mb_w * g.mb_h;
    const int bid = blockIdx.x;
    const int mbi = bid * 4 + wave;
    if (bid == 0 && threadIdx.x == 0) wave_prog[1] = 0;  // k_intra_analyze's candidate list (next kernel)
    const bool valid = mbi < nmb;
    const int mbx = valid ? mbi % g.mb_w : 0, mby = valid ? mbi / g.mb_w : 0;
    const int x0 = mbx * 16, y0 = mby * 16;
    const Planes P = planes_of(fs);
    const uint8_t* ref_uv = fs->ref_uv;
    const int cw = g.coded_w / 2, ch = g.coded_h / 2;
    int mvx = 0, mvy = 0;
    int lsad = 0;  // this lane's share of sum |luma residual| (adaptive quantisation)
    int tsad = 0;  // this lane's share of sum |src - previous src| (temporal class, aq 3)
    MbInfo mi;      // this MB's motion (16x16 or two partitions: each lane's samples use their own vector)
    mi.part = kPart16x16;
    if (valid) {
        mi = mbs[mbi];
        const int r = lane >> 2, c0 = (lane & 3) * 4;
        const Mv lv = px_mv(mi, c0, r);  // the lane's 4 luma samples lie in one partition
        mvx = lv.x;
        mvy = lv.y;
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c0);
        if (fs->aq >= 3) {
            // temporal class (h264_mb.h temporal_class): the source against the previous source,
            // displaced by the vector's integer part; this MB's source becomes the next frame's
            const int ix = mvx >> 2, iy = mvy >> 2;
            const int px = x0 + c0 + ix, py = y0 + r + iy;
            // inside the picture (no clamping): the 4 samples from one aligned dword, or two when
            // unaligned and the second stays inside the row's pitch
            if (px >= 0 && px + 4 <= g.coded_w && py >= 0 && py < g.coded_h &&
                ((px & 3) == 0 || (px & ~3) + 8 <= g.pitch)) {
                const uint32_t* qa = reinterpret_cast<const uint32_t*>(fs->prev_src + (size_t)py * g.pitch + (px & ~3));
                const uint32_t sh = (uint32_t)(px & 3);
                const uint32_t pw = sh ? __builtin_amdgcn_alignbyte(qa[1], qa[0], sh) : qa[0];
                tsad = (int)__builtin_amdgcn_sad_u8(sw, pw, 0u);
            } else {
                for (int k = 0; k < 4; ++k)
                    tsad += abs((int)((sw >> (8 * k)) & 0xff) -
                                ref_px(fs->prev_src, g.pitch, g.coded_w, g.coded_h, x0 + c0 + k + ix, y0 + r + iy));
            }
            *reinterpret_cast<uint32_t*>(fs->save_src + (y0 + r) * g.pitch + x0 + c0) = sw;
        }
        if (((mvx | mvy) & 3) == 0) {
            // full-sample vector (static desktop, scrolled text): the 4 predictions are 4 bytes of the
            // padded full-sample plane, from two aligned dwords instead of 4 byte gathers
            const uint8_t* q = P.f + (size_t)((y0 + r) + (mvy >> 2)) * P.pitch + (x0 + c0 + (mvx >> 2));
            const uint32_t* qa = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(q) & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(q) & 3);
            const uint32_t pw = sh ? __builtin_amdgcn_alignbyte(qa[1], qa[0], sh) : qa[0];
            for (int k = 0; k < 4; ++k) {
                const int p = (int)((pw >> (8 * k)) & 0xff);
                const int d = (int)((sw >> (8 * k)) & 0xff) - p;
                pred[wave][r * 16 + c0 + k] = (uint8_t)p;
                res[wave][r * 16 + c0 + k] = (int16_t)d;
                lsad += d < 0 ? -d : d;
            }
        } else {
            for (int k = 0; k < 4; ++k) {
                const int p = qpel_planes(P, (x0 + c0 + k) * 4 + mvx, (y0 + r) * 4 + mvy);
                const int d = (int)((sw >> (8 * k)) & 0xff) - p;
                pred[wave][r * 16 + c0 + k] = (uint8_t)p;
                res[wave][r * 16 + c0 + k] = (int16_t)d;
                lsad += d < 0 ? -d : d;
            }
        }
        const int cr_ = lane >> 3, cc = lane & 7;
        const int xc = x0 / 2 + cc, yc = y0 / 2 + cr_;
        const Mv cv = px_mv(mi, 2 * cc, 2 * cr_);
        for (int comp = 0; comp < 2; ++comp) {
            const int p = chroma_pred8(ref_uv, g.pitch, cw, ch, comp, xc * 8 + cv.x, yc * 8 + cv.y);
            const int sv = src_uv[yc * g.pitch + 2 * xc + comp];
            pred[wave][256 + comp * 64 + cr_ * 8 + cc] = (uint8_t)p;
            res[wave][256 + comp * 64 + cr_ * 8 + cc] = (int16_t)(sv - p);
        }
    }
    __syncthreads();
    const uint32_t lsad_mb = (uint32_t)wave_sum(lsad);
    const int tcls = temporal_class((uint32_t)wave_sum(tsad), __ballot((mvx | mvy) != 0) == 0ull);
    const int qp = mb_qp_for(fs->qp, lsad_mb, tcls, fs->aq);  // wave-uniform
    const int qpc = chroma_qp(qp, fs->chroma_qp_offset);
    int16_t* mc = coef + (size_t)(valid ? mbi : 0) * kCoefStride;

    // ---- luma: lane = 4 * blkIdx + row
    const int lb = lane >> 2, rr = lane & 3, lbx = kBlkX[lb], lby = kBlkY[lb];
    int x[4], y[4], z[4], rres[4];
    const int ro = (lby * 4 + rr) * 16 + lbx * 4;  // row offset in the MB's pred / res
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = res[wave][ro + c];
    const int hs = quad_sum(had_row_abs(x, rr));
    fdct_row(x, rr, y);
    const int nzb = quad_sum(quant_row(y, rr, qp, false, 0, z));
    {
        int d[4];
        dequant_row(z, rr, qp, d);
        idct_row(d, rr, rres);
    }
    int d_pred = 0, d_coded = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int pv = pred[wave][ro + c];
        const int e = pv + x[c] - clip255(pv + rres[c]);
        d_pred += x[c] * x[c];
        d_coded += e * e;
    }
    const uint32_t bits = rr == 0 ? block_bits_est(nzb) : 0u;
    const bool drop = valid && drop_luma_for(fs->aq, lsad_mb, tcls, qp, wave_sum(d_pred), wave_sum(d_coded),
                                             (uint32_t)wave_sum((int)bits));  // wave-uniform
    const bool drop_c = drop_chroma_for(fs->aq, tcls, drop);
    const int nz_l = drop ? 0 : nzb;
    int sse_y = 0;
    if (valid) {
        uint32_t packed = 0;
        const bool vis = x0 + lbx * 4 < g.width && (y0 + lby * 4 + rr) < g.height;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (drop) z[c] = rres[c] = 0;
            mc[kCoefLuma + lb * 16 + kZigzagInv4x4[rr * 4 + c]] = (int16_t)z[c];
            const int pv = pred[wave][ro + c];
            const int v = clip255(pv + rres[c]);
            const int e = pv + x[c] - v;
            sse_y += vis ? e * e : 0;
            packed |= (uint32_t)v << (8 * c);
        }
        *reinterpret_cast<uint32_t*>(fs->rec_y + (y0 + lby * 4 + rr) * g.pitch + x0 + lbx * 4) = packed;
        if (rr == 0) mbs[mbi].nz_luma[lby * 4 + lbx] = (uint8_t)nz_l;
    }
    const uint32_t satd_mb = (uint32_t)wave_sum(rr == 0 ? (hs + 1) >> 1 : 0);

    // ---- chroma: lanes 0..31, lane = 4 * (comp * 4 + blk) + row
    const int cbk = lane >> 2, ccomp = (cbk >> 2) & 1, cblk = cbk & 3, cbx = cblk & 1, cby = cblk >> 1;
    const int co = 256 + ccomp * 64 + (cby * 4 + rr) * 8 + cbx * 4;
    const bool clane = lane < 32;
    int cz[4], nzc = 0;
    if (clane) {
        int cx[4], cy[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) cx[c] = drop_c ? 0 : res[wave][co + c];  // a dropped MB codes no chroma residual
        fdct_row(cx, rr, cy);
        if (rr == 0) cdc[wave][ccomp * 4 + cblk] = cy[0];
        nzc = quant_row(cy, rr, qpc, false, 1, cz);
    }
    nzc = quad_sum(nzc);
    if (valid && clane) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int i = rr * 4 + c;
            if (i > 0) mc[kCoefChromaAc + (ccomp * 4 + cblk) * 16 + kZigzagInv4x4[i]] = (int16_t)cz[c];
        }
        if (rr == 0) (ccomp ? mbs[mbi].nz_cr : mbs[mbi].nz_cb)[cblk] = (uint8_t)nzc;
    }
    __syncthreads();
    if (valid && (lane == 0 || lane == 16)) {
        const int comp = lane >> 4;
        int in[4], zd[4], dq[4];
        for (int i = 0; i < 4; ++i) in[i] = cdc[wave][comp * 4 + i];
        const int n = quant_dc_chroma(in, zd, qpc, false);
        for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + comp * 4 + i] = (int16_t)zd[i];
        dequant_dc_chroma(zd, dq, qpc);
        for (int i = 0; i < 4; ++i) cdc[wave][comp * 4 + i] = dq[i];
        cdc_nz[wave][comp] = n;
    }
    __syncthreads();
    int sse_c = 0;
    if (clane) {
        int d[4], cr[4];
        dequant_row(cz, rr, qpc, d);
        if (rr == 0) d[0] = cdc[wave][ccomp * 4 + cblk];
        idct_row(d, rr, cr);
        if (valid) {
            const int xc = x0 / 2 + cbx * 4, yc = y0 / 2 + cby * 4 + rr;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int v = clip255(pred[wave][co + c] + cr[c]);
                const int e = pred[wave][co + c] + res[wave][co + c] - v;
                sse_c += (2 * (xc + c) < g.width && 2 * yc < g.height) ? e * e : 0;
                fs->rec_uv[yc * g.pitch + 2 * (xc + c) + ccomp] = (uint8_t)v;
            }
        }
    }
    {
        // Y on all lanes, U on lanes 0..15, V on 16..31
        const int sy = wave_sum(sse_y);
        const int su = wave_sum(lane < 16 ? sse_c : 0);
        const int sv = wave_sum((lane >= 16 && lane < 32) ? sse_c : 0);
        if (valid && fs->intra_in_p && lane < 3)  // per-MB copy: replaced if the MB switches to intra
            mb_sse[lane * nmb + mbi] = (uint32_t)(lane == 0 ? sy : (lane == 1 ? su : sv));
        __shared__ uint32_t part[4][4];
        if (lane == 0) {
            part[0][wave] = valid ? (uint32_t)sy : 0u;
            part[1][wave] = valid ? (uint32_t)su : 0u;
            part[2][wave] = valid ? (uint32_t)sv : 0u;
            part[3][wave] = (valid && mb_unmasked(fs, mbx, mby)) ? (uint32_t)sy : 0u;
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            const int c = threadIdx.x;
            fs->sse_part[c * kSsePartStride + bid] =
                (unsigned long long)part[c][0] + part[c][1] + part[c][2] + part[c][3];
        }
    }
    const unsigned long long luma_mask = __ballot(valid && rr == 0 && nz_l > 0);    // bit 4b: block b
    const unsigned long long chroma_mask = __ballot(valid && clane && rr == 0 && nzc > 0);
    if (valid && lane == 0) {
        int cbp = 0;
        for (int b8 = 0; b8 < 4; ++b8)
            if ((luma_mask >> (16 * b8)) & 0x1111ull) cbp |= 1 << b8;
        const int cc = (chroma_mask != 0) ? 2 : ((cdc_nz[wave][0] | cdc_nz[wave][1]) ? 1 : 0);
        cbp |= cc << 4;
        MbInfo& m = mbs[mbi];
        m.type = kMbP16x16;
        m.cbp = (uint8_t)cbp;
        m.qp = (uint8_t)qp;
        m.i16_mode = 0;
        m.chroma_mode = 0;
        m.cost = inter_cost_mb(satd_mb, fs->qp, mi);
    }
}

// ------------------------------------------------------------------ intra analysis
// raster block index -> blkIdx
__constant__ uint8_t kRasterToBlk[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per macroblock, fully parallel: SATD of the 9 Intra4x4 modes of the 16 blocks
// (144 block/mode pairs over 64 lanes), of the 4 Intra16x16 modes (one 4x4 block per lane)
// and of the 4 chroma modes, all predicted from SOURCE neighbours (open loop), then the
// shared decide_intra() on lane 0.  IDR: every MB takes its decision; P: only MBs whose
// intra cost beats the inter cost k_inter_encode left in MbInfo::cost.  Block 0 also resets
// k_intra_wave's progress counters and row ticket.
constexpr int kLT = 24;  // luma LDS tile pitch: x -1 .. 19 at columns 0 .. 20 (rows y -1 .. 15)
constexpr int kCT = 10;  // chroma LDS tile pitch (per plane): x -1 .. 7 at columns 0 .. 8
constexpr int kCTI = 20; // interleaved chroma LDS tile pitch: (x -1 .. 8) x 2 planes

__global__ __launch_bounds__(256) void k_intra_analyze(Geometry g, StateArg sa, const uint8_t* __restrict__ src_y,
                                                       const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs,
                                                       int* __restrict__ wave_prog, int32_t* __restrict__ gain,
                                                       int* __restrict__ cand) {
    __shared__ IntraCosts costs[4];
    __shared__ uint8_t ltile[4][17][kLT];   // source luma: MB + one-sample border + top-right
    __shared__ uint8_t ctile[4][9][kCTI];   // source chroma (interleaved): MB + one-sample border
    publish_state(sa);
    const FrameState* fs = &state_of(sa);
    if (blockIdx.x == 0) {
        if (!fs->idr)  // k_intra_p's per-row distortion deltas (atomically accumulated)
            for (int i = threadIdx.x; i < 4 * g.mb_h; i += 256)
                fs->sse_part[(i / g.mb_h) * kSsePartStride + (g.mb_w * g.mb_h + 3) / 4 + i % g.mb_h] = 0;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mbi = blockIdx.x * 4 + wave;
    if (mbi >= g.mb_w * g.mb_h) return;  // whole wave; no workgroup barriers below
    if (!fs->idr && !intra_candidate(mbs[mbi].cost)) {  // well-predicted: stays inter
        if (lane == 0) gain[mbi] = 0;
        return;
    }
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    const int x0 = mbx * 16, y0 = mby * 16;
    const Avail av = mb_avail(g, mbx, mby, fs->slice_rows);
    // stage the source footprint (samples outside the picture are never read: availability)
    for (int i = lane; i < 17 * 21; i += 64) {
        const int r = i / 21, cx = i - r * 21, x = x0 - 1 + cx, y = y0 - 1 + r;
        ltile[wave][r][cx] = (x >= 0 && y >= 0 && x < g.coded_w) ? src_y[y * g.pitch + x] : 0;
    }
    for (int i = lane; i < 9 * 18; i += 64) {
        const int r = i / 18, bx = i - r * 18, x = x0 - 2 + bx, y = y0 / 2 - 1 + r;
        ctile[wave][r][bx] = (x >= 0 && y >= 0) ? src_uv[y * g.pitch + x] : 0;
    }
    wave_sync_lds();
    const uint8_t* sy = &ltile[wave][1][1];
    const uint8_t* suv = &ctile[wave][1][2];
    IntraCosts& c = costs[wave];
    // lane = (4x4 block, row): every mode is evaluated by the whole wave at once (a per-lane
    // mode would diverge the prediction switch 9 ways), SATD as row Hadamards in registers plus
    // a column butterfly over the block's 4 lanes; the same integers as satd4x4().
    const int rb = lane >> 2, r = lane & 3, bx = rb & 3, by = rb >> 2;
    auto satd_quad = [&](int d0, int d1, int d2, int d3) -> uint32_t {
        int t[4] = {d0 + d1 + d2 + d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3, d0 - d1 + d2 - d3};
        uint32_t sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // column butterflies over the quad: DPP quad_perm xor 1 / xor 2
            int v = t[j];
            int o = __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
            v = (r & 1) ? o - v : v + o;
            o = __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
            v = (r & 2) ? o - v : v + o;
            sum += (uint32_t)(v < 0 ? -v : v);
        }
        sum += (uint32_t)__builtin_amdgcn_mov_dpp((int)sum, 0xB1, 0xF, 0xF, false);
        sum += (uint32_t)__builtin_amdgcn_mov_dpp((int)sum, 0x4E, 0xF, 0xF, false);
        return (sum + 1) >> 1;  // satd of the block, in all 4 lanes
    };
    {
        const Nb4 n = nb4_from_plane(sy, kLT, 0, 0, bx, by, av.left, av.top, av.topright, av.topleft);
        int sv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) sv[j] = sy[(4 * by + r) * kLT + 4 * bx + j];
        for (int m = 0; m < 9; ++m) {
            const bool ok = i4_mode_ok(m, n);
            int d[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) d[j] = ok ? sv[j] - pred4x4_px(m, n, j, r) : 0;
            const uint32_t t = satd_quad(d[0], d[1], d[2], d[3]);
            if (r == 0) c.c4[kRasterToBlk[rb]][m] = ok ? t : kCostInf;
        }
    }
    {  // Intra16x16: 4 modes, all 16 blocks at once, summed over the wave
        const NbMb n = nbmb_from_plane(sy, kLT, 0, 0, 16, 1, 0, av.left, av.top, av.topleft);
        for (int m = 0; m < 4; ++m) {
            const bool ok = i16_mode_ok(m, n);  // wave-uniform
            uint32_t t = 0;
            if (ok) {
                const PredMb p = prep_i16(m, n);
                int d[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    d[j] = (int)sy[(4 * by + r) * kLT + 4 * bx + j] - pred16_px(p, n, 4 * bx + j, 4 * by + r);
                t = satd_quad(d[0], d[1], d[2], d[3]);
                t = r == 0 ? t : 0u;
                t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x124, 0xF, 0xF, false);  // lanes l ^ 4, 8, 12
                t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x128, 0xF, 0xF, false);
                t = rows_sum(t);
            }
            if (lane == 0) c.c16[m] = ok ? t : kCostInf;
        }
    }
    {  // chroma: 4 modes; lanes 0..31 = (component, 4x4 block, row), lanes 32..63 idle
        const int comp = (lane >> 4) & 1, cb = (lane >> 2) & 3, cbx = cb & 1, cby = cb >> 1;
        const NbMb n = nbmb_from_plane(suv, kCTI, 0, 0, 8, 2, comp, av.left, av.top, av.topleft);
        for (int m = 0; m < 4; ++m) {
            const bool ok = chroma_mode_ok(m, n);  // wave-uniform (same availability for both planes)
            uint32_t t = 0;
            if (ok) {
                const PredMb p = prep_chroma(m, n);
                int d[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    d[j] = lane < 32 ? (int)suv[(4 * cby + r) * kCTI + 2 * (4 * cbx + j) + comp] -
                                           predc_px(p, n, 4 * cbx + j, 4 * cby + r)
                                     : 0;
                t = satd_quad(d[0], d[1], d[2], d[3]);
                t = (r == 0 && lane < 32) ? t : 0u;
                t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x124, 0xF, 0xF, false);  // lanes l ^ 4, 8, 12
                t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x128, 0xF, 0xF, false);
                t = rows_sum(t);
            }
            if (lane == 0) c.cc[m] = ok ? t : kCostInf;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
        const IntraDecision d = decide_intra(c, fs->qp, fs->intra4x4 != 0);
        MbInfo& m = mbs[mbi];
        const int32_t gn = fs->idr ? 1 : intra_gain(d.cost_luma, m.cost, fs->qp);
        if (!fs->idr) {
            gain[mbi] = gn;
            if (gn > 0) cand[atomicAdd(&wave_prog[1], 1)] = mbi;  // k_intra_p's work list
        }
        if (gn > 0) {  // IDR: the decision; P: a pending decision, applied by k_intra_p if selected
            const int qp = fs->qp;
            if (fs->idr)
                m.type = (uint8_t)d.type;
            else
                m.itype = (uint8_t)d.type;
            m.i16_mode = (uint8_t)d.i16_mode;
            m.chroma_mode = (uint8_t)d.chroma_mode;
            uint8_t md[8];
            for (int rb = 0; rb < 16; rb += 2) md[rb >> 1] = (uint8_t)(d.i4[rb] | (d.i4[rb + 1] << 4));
            for (int k = 0; k < 8; ++k) m.i4[k] = md[k];
            if (fs->idr) {
                m.qp = (uint8_t)qp;
                m.mvx = 0;
                m.mvy = 0;
            }
        }
    }
}

// ------------------------------------------------------------------ intra reconstruction
// Closed-loop coding of the intra macroblocks in a diagonal wavefront.  One workgroup per MB
// row (row order taken from a ticket counter, so a row only ever waits on rows that are
// already running); wave 0 codes luma, wave 1 chroma -- the two planes' intra predictions
// are independent, so they run as two wavefronts.  A macroblock waits until the row above
// (same slice) has finished the macroblock above-right (per-plane progress counters,
// agent-scope release / acquire).  Neighbour samples are staged in LDS tiles with a one-
// sample border; the prediction helpers read them through the same plane-accessors as the
// CPU encoder, so decisions and reconstructions are bit-identical.
//  * Intra4x4: the 16 blocks in 10 dependency steps (block (bx,by) at step bx + 2*by, up to
//    two blocks per step), one pixel per lane; the 4x4 transforms run as row / column
//    butterflies over lane shuffles within each 16-lane block group.
//  * Intra16x16 and chroma: one 4x4 block per lane, DC transforms on one lane.
// In P pictures the waves skip inter macroblocks (final since k_inter_encode) and replace the
// inter distortion of the switched macroblocks by a per-row delta partial.


// Per-MB fields the reconstruction needs, read once (prefetched a macroblock ahead).
struct MbFields {
    int type, qp, i16_mode, chroma_mode;
    uint32_t i4lo, i4hi;  // Intra4x4 modes, nibbles in raster block order
    __device__ int i4(int rb) const { return (int)(((rb < 8 ? i4lo : i4hi) >> (4 * (rb & 7))) & 15u); }
};
__device__ __forceinline__ MbFields load_fields(const MbInfo* m) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(m);  // MbInfo: 48 B, dword aligned
    const uint32_t d1 = w[1], d8 = w[8], d9 = w[9], d10 = w[10];
    MbFields f;
    f.type = (int)(d1 & 0xff);
    f.i16_mode = (int)((d1 >> 16) & 0xff);
    f.chroma_mode = (int)(d1 >> 24);
    f.qp = (int)((d8 >> 8) & 0xff);
    f.i4lo = d9;
    f.i4hi = d10;
    return f;
}
static_assert(offsetof(MbInfo, type) == 4 && offsetof(MbInfo, i16_mode) == 6 && offsetof(MbInfo, chroma_mode) == 7 &&
                  offsetof(MbInfo, qp) == 33 && offsetof(MbInfo, i4) == 36,
              "load_fields() layout");


// Quantiser constants of one QP, read with wave-uniform indices (scalar loads) and picked per
// coefficient position with selects: a lane-indexed table read is a vector memory round trip,
// and in the wavefront every one of them sits on the critical path (profiles/r02_idr).
struct QpTab {
    int mf0, mf1, mf2;  // kQuantMF[qp % 6][class]
    int dv0, dv1, dv2;  // kDequantV[qp % 6][class]
    int qbits, qs;
    uint32_t f_intra;
    __device__ int mf(int cls) const { return cls == 0 ? mf0 : (cls == 1 ? mf1 : mf2); }
    __device__ int dv(int cls) const { return cls == 0 ? dv0 : (cls == 1 ? dv1 : dv2); }
};
__device__ __forceinline__ QpTab qp_tab(int qp) {
    QpTab t;
    const int qm = qp % 6;
    t.mf0 = kQuantMF[qm][0];
    t.mf1 = kQuantMF[qm][1];
    t.mf2 = kQuantMF[qm][2];
    t.dv0 = kDequantV[qm][0];
    t.dv1 = kDequantV[qm][1];
    t.dv2 = kDequantV[qm][2];
    t.qbits = 15 + qp / 6;
    t.qs = qp / 6;
    t.f_intra = (1u << t.qbits) / 3;
    return t;
}
// kPosClass of raster position (r, c): 0 both even, 1 both odd, 2 mixed
__device__ __forceinline__ int pos_class(int r, int c) { return ((r | c) & 1) == 0 ? 0 : (((r & c) & 1) ? 1 : 2); }
// kZigzagInv4x4 as nibbles of one 64-bit immediate
constexpr uint64_t zz_inv_packed() {
    uint64_t v = 0;
    for (int i = 0; i < 16; ++i) v |= (uint64_t)kZigzagInv4x4[i] << (4 * i);
    return v;
}
__device__ __forceinline__ int zz_inv(int i) { return (int)((zz_inv_packed() >> (4 * i)) & 15u); }
// blkIdx <-> raster 4x4 block position (6.4.3), arithmetic
__device__ __forceinline__ int blk_x(int b) { return (b & 1) | ((b >> 1) & 2); }
__device__ __forceinline__ int blk_y(int b) { return ((b >> 1) & 1) | ((b >> 2) & 2); }
// Intra4x4 schedule: raster block of quad group `grp` (0, 1) at dependency step t (block
// (bx, by) at step bx + 2 by), -1 if none
__device__ __forceinline__ int i4_step_block(int t, int grp) {
    const int by = (t >= 2 ? (t - 2) >> 1 : 0) + grp, bx = t - 2 * by;
    return (bx >= 0 && bx <= 3 && by <= 3) ? by * 4 + bx : -1;
}
__device__ __forceinline__ int raster_to_blk(int rb) {
    const int bx = rb & 3, by = rb >> 2;
    return ((by >> 1) << 3) | ((bx >> 1) << 2) | ((by & 1) << 1) | (bx & 1);
}
// quant4x4 / dequant4x4 of row r (intra rounding), 32-bit: |y| * MF + f < 2^31 for 8-bit video
__device__ __forceinline__ int quant_row_i(const int* y, int r, const QpTab& t, int start, int* z) {
    int nz = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int a = y[c] < 0 ? -y[c] : y[c];
        int q = (int)(((uint32_t)a * (uint32_t)t.mf(pos_class(r, c)) + t.f_intra) >> t.qbits);
        q = q > kMaxLevel ? kMaxLevel : q;
        q = (r * 4 + c) < start ? 0 : q;
        z[c] = y[c] < 0 ? -q : q;
        nz += (q != 0);
    }
    return nz;
}
__device__ __forceinline__ void dequant_row_t(const int* z, int r, const QpTab& t, int* d) {
#pragma unroll
    for (int c = 0; c < 4; ++c) d[c] = z[c] * t.dv(pos_class(r, c)) * (1 << t.qs);
}
// Hadamard of row r of a 4x4 block whose rows sit in the quad (hadamard4x4, rows then columns)
__device__ __forceinline__ void had_row(const int* x, int r, int* y) {
    const int t[4] = {x[0] + x[1] + x[2] + x[3], x[0] + x[1] - x[2] - x[3], x[0] - x[1] - x[2] + x[3],
                      x[0] - x[1] + x[2] - x[3]};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int a = qbc<0>(t[c]), b = qbc<1>(t[c]), cc = qbc<2>(t[c]), d = qbc<3>(t[c]);
        y[c] = r == 0 ? a + b + cc + d : r == 1 ? a + b - cc - d : r == 2 ? a - b - cc + d : a - b + cc - d;
    }
}

// The 4 prediction samples of row r of an Intra4x4 block: one switch on the mode per row
// (the per-sample pred4x4_px switch, unrolled over the row, evaluated 4 mode switches with
// the quads' different modes as divergent branch chains); same formulas, constant-folded.
template <int M>
__device__ __forceinline__ void pred4x4_row_m(const Nb4& n, int r, int* pv) {
#pragma unroll
    for (int c = 0; c < 4; ++c) pv[c] = pred4x4_px(M, n, c, r);
}
__device__ __forceinline__ void pred4x4_row(int mode, const Nb4& n, int r, int* pv) {
    switch (mode) {
        case 0: pred4x4_row_m<0>(n, r, pv); break;
        case 1: pred4x4_row_m<1>(n, r, pv); break;
        case 2: pred4x4_row_m<2>(n, r, pv); break;
        case 3: pred4x4_row_m<3>(n, r, pv); break;
        case 4: pred4x4_row_m<4>(n, r, pv); break;
        case 5: pred4x4_row_m<5>(n, r, pv); break;
        case 6: pred4x4_row_m<6>(n, r, pv); break;
        case 7: pred4x4_row_m<7>(n, r, pv); break;
        default: pred4x4_row_m<8>(n, r, pv); break;
    }
}

// Intra16x16 / chroma prediction of 4 samples of one row, the mode switch hoisted out of the row
template <int M, bool C>
__device__ __forceinline__ void predmb_row_m(const PredMb& p, const NbMb& n, int x0, int y, int* pv) {
    PredMb q = p;
    q.mode = M;  // constant mode: the helpers' switches fold
#pragma unroll
    for (int c = 0; c < 4; ++c) pv[c] = C ? predc_px(q, n, x0 + c, y) : pred16_px(q, n, x0 + c, y);
}
template <bool C>
__device__ __forceinline__ void predmb_row(const PredMb& p, const NbMb& n, int x0, int y, int* pv) {
    switch (p.mode) {
        case 0: predmb_row_m<0, C>(p, n, x0, y, pv); break;
        case 1: predmb_row_m<1, C>(p, n, x0, y, pv); break;
        case 2: predmb_row_m<2, C>(p, n, x0, y, pv); break;
        default: predmb_row_m<3, C>(p, n, x0, y, pv); break;
    }
}

// One Intra4x4 block on a quad (row r on this lane): predict from the tile, transform,
// quantise, store the levels, reconstruct into the tile.  Returns the block's level count.
__device__ __forceinline__ int i4_code_block(const Geometry& g, int rb, int r, int mode, const QpTab& T,
                                             const uint32_t* ls, uint8_t (*lt)[kLT], int16_t* __restrict__ mc, int x0,
                                             int y0, const Avail& av, uint32_t& sse) {
    const uint8_t* tile = &lt[1][1];
    const int bx = rb & 3, by = rb >> 2, py = 4 * by + r;
    const Nb4 n = nb4_from_plane(tile, kLT, 0, 0, bx, by, av.left, av.top, av.topright, av.topleft);
    const uint32_t sw = ls[py * 4 + bx];
    int pv[4], x[4], y[4], z[4], d[4], rr[4];
    pred4x4_row(mode, n, r, pv);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = (int)((sw >> (8 * c)) & 0xff) - pv[c];
    fdct_row(x, r, y);
    const int nzb = quad_sum(quant_row_i(y, r, T, 0, z));
    const int b = raster_to_blk(rb);
#pragma unroll
    for (int c = 0; c < 4; ++c) mc[kCoefLuma + b * 16 + zz_inv(r * 4 + c)] = (int16_t)z[c];
    dequant_row_t(z, r, T, d);
    idct_row(d, r, rr);
    const bool vis = y0 + py < g.height;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int rec = clip255(pv[c] + rr[c]);
        lt[1 + py][1 + 4 * bx + c] = (uint8_t)rec;
        const int e = x[c] + pv[c] - rec;
        sse += (vis && x0 + 4 * bx + c < g.width) ? (uint32_t)(e * e) : 0u;
    }
    return nzb;
}

// Closed-loop coding of one intra macroblock's luma, in the 4x4 "row" layout of
// k_inter_encode (lane 4b + r = row r of block b): every transform pass is in-lane or a DPP
// quad broadcast, the quantiser tables are scalar.  ls: the MB's source luma (16 rows x 4
// dwords); lt: the LDS tile with the neighbours at row 0 / column 0, reconstructed in place.
//  * Intra4x4: the 16 blocks in 10 dependency steps (block (bx,by) at step bx + 2*by, up to
//    two blocks = two quads per step).
//  * Intra16x16: all 16 blocks at once; the DC Hadamard / quantiser on quad 0 (row layout of
//    the 4x4 DC matrix).
__device__ void intra_luma_mb(const Geometry& g, const MbFields& f, const uint32_t* ls, MbInfo& m,
                              int16_t* __restrict__ mc, int mbx, int mby, const Avail& av, uint8_t (*lt)[kLT],
                              int* ldc, int lane, uint32_t& sse) {
    const int x0 = mbx * 16, y0 = mby * 16;
    const QpTab T = qp_tab(f.qp);
    const uint8_t* tile = &lt[1][1];
    const int r = lane & 3;
    int cbp_l = 0;
    if (f.type == kMbI4x4) {
        const int grp = lane >> 2;
        for (int t = 0; t < 10; ++t) {
            const int rb = grp < 2 ? i4_step_block(t, grp) : -1;  // uniform per quad
            int nzb = 0;
            if (rb >= 0) {
                nzb = i4_code_block(g, rb, r, f.i4(rb), T, ls, lt, mc, x0, y0, av, sse);
                if (r == 0) m.nz_luma[rb] = (uint8_t)nzb;
            }
            const unsigned long long any = __ballot(rb >= 0 && r == 0 && nzb > 0);
            for (int gq = 0; gq < 2; ++gq)
                if ((any >> (4 * gq)) & 1ull) cbp_l |= 1 << (raster_to_blk(i4_step_block(t, gq)) >> 2);
            wave_sync_lds();
        }
    } else {  // Intra16x16
        const NbMb n = nbmb_from_plane(tile, kLT, 0, 0, 16, 1, 0, av.left, av.top, av.topleft);
        const PredMb p = prep_i16(f.i16_mode, n);
        const int b = lane >> 2, bx = blk_x(b), by = blk_y(b), py = 4 * by + r;
        const uint32_t sw = ls[py * 4 + bx];
        int pv[4], x[4], y[4], z[4];
        predmb_row<false>(p, n, 4 * bx, py, pv);
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = (int)((sw >> (8 * c)) & 0xff) - pv[c];
        fdct_row(x, r, y);
        if (r == 0) ldc[by * 4 + bx] = y[0];
        const int nz = quad_sum(quant_row_i(y, r, T, 1, z));
#pragma unroll
        for (int c = 0; c < 4; ++c) mc[kCoefLuma + b * 16 + zz_inv(r * 4 + c)] = (int16_t)z[c];
        wave_sync_lds();
        if (lane < 4) {  // DC matrix row `lane`: Hadamard, /2, quantise (quant_dc_luma), then dequant_dc_luma
            int dc[4], h[4], zd[4], fh[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) dc[c] = ldc[lane * 4 + c];
            had_row(dc, lane, h);
            const uint32_t qb = (uint32_t)(T.qbits + 1), fd = 2u * ((1u << (qb - 1)) / 3);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int v = h[c] >> 1;
                const int a = v < 0 ? -v : v;
                int q = (int)(((uint32_t)a * (uint32_t)T.mf0 + fd) >> qb);
                q = q > kMaxLevel ? kMaxLevel : q;
                zd[c] = v < 0 ? -q : q;
                mc[kCoefLumaDc + zz_inv(lane * 4 + c)] = (int16_t)zd[c];
            }
            had_row(zd, lane, fh);
            const int ls16 = 16 * T.dv0;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                ldc[lane * 4 + c] = f.qp >= 36 ? fh[c] * ls16 * (1 << (T.qs - 6))
                                               : (fh[c] * ls16 + (1 << (5 - T.qs))) >> (6 - T.qs);
        }
        wave_sync_lds();
        const bool luma_ac = __ballot(r == 0 && nz > 0) != 0;
        int d[4], rr[4];
        dequant_row_t(z, r, T, d);
        if (r == 0) d[0] = ldc[by * 4 + bx];
        idct_row(d, r, rr);
        const bool vis = y0 + py < g.height;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int rec = clip255(pv[c] + rr[c]);
            lt[1 + py][1 + 4 * bx + c] = (uint8_t)rec;
            const int e = x[c] + pv[c] - rec;
            sse += (vis && x0 + 4 * bx + c < g.width) ? (uint32_t)(e * e) : 0u;
        }
        if (r == 0) m.nz_luma[by * 4 + bx] = (uint8_t)(luma_ac ? nz : 0);
        cbp_l = luma_ac ? 15 : 0;
        wave_sync_lds();
    }
    if (lane == 0) m.cbp = (uint8_t)cbp_l;  // chroma bits merged at the end of the row
}

// Chroma of one intra macroblock, row layout on lanes 0..31 (lane 4 (comp * 4 + blk) + r).
// cs: the MB's source chroma (8 rows x 4 dwords of interleaved Cb/Cr).
__device__ void intra_chroma_mb(const Geometry& g, int chroma_qp_offset, const MbFields& f, const uint32_t* cs,
                                MbInfo& m, int16_t* __restrict__ mc, int mbx, int mby, const Avail& av,
                                uint8_t (*ct)[9][kCT], int* cdc, int lane, uint32_t& sse_u, uint32_t& sse_v) {
    const int xc0 = mbx * 8, yc0 = mby * 8;
    const int qpc = chroma_qp(f.qp, chroma_qp_offset);
    const QpTab T = qp_tab(qpc);
    const int r = lane & 3, cbk = (lane >> 2) & 7, comp = cbk >> 2, cb = cbk & 3, bx = cb & 1, by = cb >> 1;
    const int py = 4 * by + r;
    const bool clane = lane < 32;
    int pv[4] = {0, 0, 0, 0}, x[4] = {0, 0, 0, 0}, z[4] = {0, 0, 0, 0}, nz = 0;
    if (clane) {
        const NbMb n = nbmb_from_plane(&ct[comp][1][1], kCT, 0, 0, 8, 1, 0, av.left, av.top, av.topleft);
        const PredMb p = prep_chroma(f.chroma_mode, n);
        // samples 4bx .. 4bx+3 of this plane = bytes 8bx + 2c + comp of the interleaved row
        const uint32_t w0 = cs[py * 4 + 2 * bx], w1 = cs[py * 4 + 2 * bx + 1];
        int y[4];
        predmb_row<true>(p, n, 4 * bx, py, pv);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t w = c < 2 ? w0 : w1;
            x[c] = (int)((w >> (8 * (2 * (c & 1) + comp))) & 0xff) - pv[c];
        }
        fdct_row(x, r, y);
        if (r == 0) cdc[comp * 4 + cb] = y[0];
        nz = quad_sum(quant_row_i(y, r, T, 1, z));
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (r * 4 + c > 0) mc[kCoefChromaAc + (comp * 4 + cb) * 16 + zz_inv(r * 4 + c)] = (int16_t)z[c];
        if (r == 0) (comp ? m.nz_cr : m.nz_cb)[cb] = (uint8_t)nz;
    }
    wave_sync_lds();
    int ndc = 0;
    if (lane == 0 || lane == 16) {
        const int cp = lane >> 4;
        int in[4], zd[4], dq[4];
        for (int i = 0; i < 4; ++i) in[i] = cdc[cp * 4 + i];
        ndc = quant_dc_chroma(in, zd, qpc, true);
        for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + cp * 4 + i] = (int16_t)zd[i];
        dequant_dc_chroma(zd, dq, qpc);
        for (int i = 0; i < 4; ++i) cdc[cp * 4 + i] = dq[i];
    }
    wave_sync_lds();
    const bool any_ac = __ballot(clane && nz > 0) != 0, any_dc = __ballot(ndc > 0) != 0;
    if (clane) {
        int d[4], rr[4];
        dequant_row_t(z, r, T, d);
        if (r == 0) d[0] = cdc[comp * 4 + cb];
        idct_row(d, r, rr);
        uint32_t s = 0;
        const bool vis = 2 * (yc0 + py) < g.height;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int xc = xc0 + 4 * bx + c;
            const int rec = clip255(pv[c] + rr[c]);
            const int e = x[c] + pv[c] - rec;
            s += (vis && 2 * xc < g.width) ? (uint32_t)(e * e) : 0u;
            ct[comp][1 + py][1 + 4 * bx + c] = (uint8_t)rec;
        }
        if (comp)
            sse_v += s;
        else
            sse_u += s;
    }
    if (lane == 0) m.cbp_c = (uint8_t)(any_ac ? 2 : (any_dc ? 1 : 0));
    wave_sync_lds();
}


// IDR reconstruction: one workgroup per (slice, plane) -- every MB row of the slice is one wave
// of the workgroup (idr_slice_rows() <= 8), luma and chroma are separate workgroups (the two
// planes' intra predictions are independent).  The diagonal wavefront's row-to-row hand-off
// stays inside the CU: a row publishes each macroblock's bottom sample line into an LDS line
// buffer and then its progress counter; the row below waits on that counter (luma: the MB
// above-right, chroma: the MB above).  LDS operations of one wave complete in issue order,
// so a reader that sees the counter sees the line.  The cross-CU version of this hand-off
// (tagged L2-bypassing line words between per-row workgroups) spent most of its time waiting
// for the stores to become visible (profiles/r02_idr).
struct IntraWaveTiles {
    uint8_t lt[17][kLT];    // luma tile: row 0 = top neighbours, column 0 = left neighbours
    uint8_t ct[2][9][kCT];  // chroma tiles (Cb, Cr)
    uint32_t src[64];       // source of the current MB (luma 16 x 16 / chroma 8 rows x 16 bytes)
    int dc[16];             // luma DC / chroma DC scratch
};

// One plane's rows of the slice.
template <bool chroma>
__device__ __forceinline__ void intra_wave_rows(const Geometry& g, const FrameState* __restrict__ fs,
                                             const uint8_t* __restrict__ src_y, const uint8_t* __restrict__ src_uv,
                                             MbInfo* __restrict__ mbs, int16_t* __restrict__ coef, uint8_t* s_line,
                                             IntraWaveTiles* tiles, int* prog) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slice_rows = fs->slice_rows, cqp_off = fs->chroma_qp_offset;
    uint8_t* const rec_y = fs->rec_y;
    uint8_t* const rec_uv = fs->rec_uv;
    const int mby = blockIdx.x * slice_rows + wave;
    const bool active = mby < g.mb_h;  // the last slice may be shorter (whole waves)
    if (!active) return;  // no workgroup barriers below
    IntraWaveTiles& T = tiles[wave];
    uint8_t* my_line = s_line + (size_t)wave * g.coded_w;
    const uint8_t* up_line = s_line + (size_t)(wave > 0 ? wave - 1 : 0) * g.coded_w;
    uint32_t sse_a = 0, sse_b = 0;  // luma: Y; chroma: U, V
    uint32_t sse_m = 0;             // luma: Y of the MBs outside the quality-report mask
    // software pipeline: the next MB's source dword and fields load while this one is coded
    auto fetch_src = [&](int mbx) -> uint32_t {
        if (mbx >= g.mb_w) return 0u;
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        if (!chroma) return *reinterpret_cast<const uint32_t*>(src_y + (size_t)(mby * 16 + r) * g.pitch + mbx * 16 + c4);
        if (lane >= 32) return 0u;
        return *reinterpret_cast<const uint32_t*>(src_uv + (size_t)(mby * 8 + r) * g.pitch + mbx * 16 + c4);
    };
    uint32_t nsrc = fetch_src(0);
    MbFields nf = load_fields(&mbs[mby * g.mb_w]);
#ifdef MX_IDR_TIMING
    const unsigned long long t_start = wall_clock64();
#endif
    for (int mbx = 0; mbx < g.mb_w; ++mbx) {
        const int mbi = mby * g.mb_w + mbx;
        MbInfo& m = mbs[mbi];
        const MbFields f = nf;
        T.src[lane] = nsrc;
        nsrc = fetch_src(mbx + 1);
        nf = load_fields(&mbs[mby * g.mb_w + (mbx + 1 < g.mb_w ? mbx + 1 : mbx)]);
        const Avail av = mb_avail(g, mbx, mby, slice_rows);
        int16_t* mc = coef + (size_t)mbi * kCoefStride;
        if (av.top) {  // wait for the row above (uniform)
            const int need = chroma ? mbx + 1 : (av.topright ? mbx + 2 : mbx + 1);
            while (__hip_atomic_load(&prog[wave - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
                __builtin_amdgcn_s_sleep(1);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
        }
        if (!chroma) {
            const int x0 = mbx * 16, y0 = mby * 16;
            // the left column is the previous MB's right column, already in the tile
            const uint8_t keep = lane < 16 ? T.lt[1 + lane][16] : 0;
            const int x = x0 - 1 + lane;
            const bool need = lane < 21 && (lane == 0 ? av.topleft : (lane <= 16 ? av.top : av.topright));
            const uint8_t top = need ? up_line[x] : 0;
            wave_sync_lds();
            if (lane < 16) T.lt[1 + lane][0] = av.left ? keep : 0;
            if (lane < 21) T.lt[0][lane] = top;
            wave_sync_lds();
            uint32_t sse_mb = 0;
            intra_luma_mb(g, f, T.src, m, mc, mbx, mby, av, T.lt, T.dc, lane, sse_mb);
            sse_a += sse_mb;
            if (mb_unmasked(fs, mbx, mby)) sse_m += sse_mb;
            // tile -> reconstruction: 16 rows x 16 bytes, one dword per lane; bottom line -> LDS
            const int r = lane >> 2, c4 = (lane & 3) * 4;
            const uint32_t v = (uint32_t)T.lt[1 + r][1 + c4] | ((uint32_t)T.lt[1 + r][2 + c4] << 8) |
                               ((uint32_t)T.lt[1 + r][3 + c4] << 16) | ((uint32_t)T.lt[1 + r][4 + c4] << 24);
            *reinterpret_cast<uint32_t*>(rec_y + (size_t)(y0 + r) * g.pitch + x0 + c4) = v;
            if (r == 15) *reinterpret_cast<uint32_t*>(my_line + x0 + c4) = v;
        } else {
            const int xc0 = mbx * 8, yc0 = mby * 8;
            uint8_t keep = 0;
            if (lane < 16) keep = T.ct[lane >> 3][1 + (lane & 7)][8];
            // top: lanes 16..33 -> (comp, cx 0..8 = x -1..7), byte 2*(xc0-1+cx)+comp of the line
            const int k = lane - 16, comp_t = k >= 9 ? 1 : 0, cx = k - 9 * comp_t;
            const int x = 2 * (xc0 - 1 + cx) + comp_t;
            const bool need = lane >= 16 && lane < 34 && (cx == 0 ? av.topleft : av.top);
            const uint8_t top = need ? up_line[x] : 0;
            wave_sync_lds();
            if (lane < 16)
                T.ct[lane >> 3][1 + (lane & 7)][0] = av.left ? keep : 0;
            else if (lane < 34)
                T.ct[comp_t][0][cx] = top;
            wave_sync_lds();
            intra_chroma_mb(g, cqp_off, f, T.src, m, mc, mbx, mby, av, T.ct, T.dc, lane, sse_a, sse_b);
            if (lane < 32) {  // 8 rows x 16 interleaved bytes, one dword (2 samples x 2 planes) per lane
                const int r = lane >> 2, c2 = (lane & 3) * 2;
                const uint32_t v = (uint32_t)T.ct[0][1 + r][1 + c2] | ((uint32_t)T.ct[1][1 + r][1 + c2] << 8) |
                                   ((uint32_t)T.ct[0][1 + r][2 + c2] << 16) | ((uint32_t)T.ct[1][1 + r][2 + c2] << 24);
                *reinterpret_cast<uint32_t*>(rec_uv + (size_t)(yc0 + r) * g.pitch + 2 * (xc0 + c2)) = v;
                if (r == 7) *reinterpret_cast<uint32_t*>(my_line + 2 * (xc0 + c2)) = v;
            }
        }
        // publish: the line stores above were issued first, and LDS completes them in order
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (lane == 0) __hip_atomic_store(&prog[wave], mbx + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
#ifdef MX_IDR_TIMING
    if (lane == 0)
        printf("MXIDR plane %d slice %d row %d wall_ticks %llu\n", (int)chroma, (int)blockIdx.x, wave, wall_clock64() - t_start);
#endif
    // distortion of the row (one partial per row and channel)
    unsigned long long a = sse_a, b = sse_b, mm = sse_m;
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
        mm += __shfl_xor(mm, o, 64);
    }
    if (lane == 0) {
        if (!chroma) {
            fs->sse_part[0 * kSsePartStride + mby] = a;
            fs->sse_part[3 * kSsePartStride + mby] = mm;
        } else {
            fs->sse_part[1 * kSsePartStride + mby] = a;
            fs->sse_part[2 * kSsePartStride + mby] = b;
        }
    }
}

// Luma rows with consecutive Intra4x4 macroblocks pipelined: block (bx, by) of the k-th MB of
// a run of Intra4x4 MBs runs at step 4k + bx + 2by.  Its left neighbours (block (3, by) of
// MB k-1, step 4k - 1 + 2by) and top-left are done a step earlier, and the predecessor copies
// each finished right-column block into the successor's tile; so up to three MBs are in
// flight (one quad pair each, lanes 8j .. 8j+7 for tile slot j = mbx % 3) and a run of n
// such MBs takes 4n + 6 dependent steps instead of 10n.  Intra16x16 MBs (the whole MB's DC
// transform couples all blocks) are coded alone between runs.  The IDR picture QP is
// uniform (k_intra_analyze), so one quantiser table serves every MB in flight.
struct LumaPipeTiles {
    uint8_t lt[3][17][kLT];  // tile slot mbx % 3: row 0 = top neighbours, column 0 = left neighbours
    uint32_t src[3][64];     // the slot MB's source (16 rows x 4 dwords)
    int dc[16];              // Intra16x16 DC scratch
};

__device__ __forceinline__ void intra_luma_rows_pl(const Geometry& g, const FrameState* __restrict__ fs,
                                                   const uint8_t* __restrict__ src_y, MbInfo* __restrict__ mbs,
                                                   int16_t* __restrict__ coef, uint8_t* s_line, LumaPipeTiles* tiles,
                                                   int* prog) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slice_rows = fs->slice_rows;
    uint8_t* const rec_y = fs->rec_y;
    const int mby = blockIdx.x * slice_rows + wave;
    if (mby >= g.mb_h) return;  // the last slice may be shorter (whole waves); no barriers below
    LumaPipeTiles& P = tiles[wave];
    uint8_t* my_line = s_line + (size_t)wave * g.coded_w;
    const uint8_t* up_line = s_line + (size_t)(wave > 0 ? wave - 1 : 0) * g.coded_w;
    const int y0 = mby * 16;
    const QpTab T = qp_tab(fs->qp);
    uint32_t sse_a = 0, sse_m = 0;
    auto fetch_src = [&](int mbx) -> uint32_t {
        if (mbx >= g.mb_w) return 0u;
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        return *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y0 + r) * g.pitch + mbx * 16 + c4);
    };
    uint32_t nsrc = fetch_src(0);
    MbFields nf = load_fields(&mbs[mby * g.mb_w]);
    // stage MB x into its slot: source, top neighbours (after the row above published them) and,
    // if `left`, the left column from the completed previous MB's slot
    auto stage = [&](int x, bool left) {
        const int j = x % 3;
        P.src[j][lane] = nsrc;
        nsrc = fetch_src(x + 1);
        const Avail av = mb_avail(g, x, mby, slice_rows);
        if (av.top) {
            const int need = av.topright ? x + 2 : x + 1;
            while (__hip_atomic_load(&prog[wave - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
                __builtin_amdgcn_s_sleep(1);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
        }
        const bool need = lane < 21 && (lane == 0 ? av.topleft : (lane <= 16 ? av.top : av.topright));
        const uint8_t top = need ? up_line[x * 16 - 1 + lane] : 0;
        uint8_t lft = 0;
        if (left && lane < 16 && av.left) lft = P.lt[(x + 2) % 3][1 + lane][16];
        wave_sync_lds();
        if (lane < 21) P.lt[j][0][lane] = top;
        if (left && lane < 16) P.lt[j][1 + lane][0] = lft;
        wave_sync_lds();
    };
    // MB x is complete: tile -> reconstruction, bottom line -> LDS, then publish it
    auto finish = [&](int x) {
        const int j = x % 3, x0 = x * 16;
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        const uint32_t v = (uint32_t)P.lt[j][1 + r][1 + c4] | ((uint32_t)P.lt[j][1 + r][2 + c4] << 8) |
                           ((uint32_t)P.lt[j][1 + r][3 + c4] << 16) | ((uint32_t)P.lt[j][1 + r][4 + c4] << 24);
        *reinterpret_cast<uint32_t*>(rec_y + (size_t)(y0 + r) * g.pitch + x0 + c4) = v;
        if (r == 15) *reinterpret_cast<uint32_t*>(my_line + x0 + c4) = v;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // LDS completes the line stores before the counter
        if (lane == 0) __hip_atomic_store(&prog[wave], x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
#ifdef MX_IDR_TIMING
    const unsigned long long t_start = wall_clock64();
#endif
    int next = 0;  // next MB to start
    while (next < g.mb_w) {
        if (nf.type != kMbI4x4) {  // Intra16x16: alone
            const int x = next;
            const MbFields f = nf;
            nf = load_fields(&mbs[mby * g.mb_w + (x + 1 < g.mb_w ? x + 1 : x)]);
            stage(x, true);
            const int j = x % 3, mbi = mby * g.mb_w + x;
            uint32_t sse_mb = 0;
            intra_luma_mb(g, f, P.src[j], mbs[mbi], coef + (size_t)mbi * kCoefStride, x, mby,
                          mb_avail(g, x, mby, slice_rows), P.lt[j], P.dc, lane, sse_mb);
            sse_a += sse_mb;
            if (mb_unmasked(fs, x, mby)) sse_m += sse_mb;
            finish(x);
            ++next;
            continue;
        }
        // a run of Intra4x4 MBs from `base`; MB base + k starts at step 4k while the run lasts
        const int base = next;
        int started = 0;
        bool open = true;
        uint32_t mlo[3] = {0, 0, 0}, mhi[3] = {0, 0, 0};  // Intra4x4 modes per slot (uniform)
        int cbp[3] = {0, 0, 0};
        int sk[3] = {-16, -16, -16};      // run index k of the MB in each slot (uniform)
        bool um[3] = {false, false, false};  // the slot MB counts towards the masked PSNR
        for (int t = 0;; ++t) {
            if ((t & 3) == 0 && open) {
                if (base + started < g.mb_w && nf.type == kMbI4x4) {
                    const int x = base + started, j = x % 3;
                    const MbFields f = nf;
                    nf = load_fields(&mbs[mby * g.mb_w + (x + 1 < g.mb_w ? x + 1 : x)]);
                    const bool unm = mb_unmasked(fs, x, mby);
#pragma unroll
                    for (int s = 0; s < 3; ++s)
                        if (s == j) {
                            mlo[s] = f.i4lo;
                            mhi[s] = f.i4hi;
                            cbp[s] = 0;
                            sk[s] = started;
                            um[s] = unm;
                        }
                    stage(x, started == 0);  // later MBs get their left column from the predecessor
                    ++started;
                } else {
                    open = false;
                }
            }
            if (!open && t > 4 * (started - 1) + 9) break;
            // this lane's MB (slot j = lane / 8, quad group grp) and its local step
            const int j = lane >> 3, grp = (lane >> 2) & 1, r = lane & 3;
            const int k = j == 0 ? sk[0] : (j == 1 ? sk[1] : sk[2]);
            const int sl = t - 4 * k;
            const bool mine = lane < 24 && k >= 0 && sl <= 9;
            const int rb = mine ? i4_step_block(sl, grp) : -1;  // uniform per quad
            int nzb = 0;
            if (rb >= 0) {
                const int x = base + k, mbi = mby * g.mb_w + x;
                const uint32_t lo = j == 0 ? mlo[0] : (j == 1 ? mlo[1] : mlo[2]);
                const uint32_t hi = j == 0 ? mhi[0] : (j == 1 ? mhi[1] : mhi[2]);
                const int mode = (int)(((rb < 8 ? lo : hi) >> (4 * (rb & 7))) & 15u);
                uint32_t e2 = 0;
                nzb = i4_code_block(g, rb, r, mode, T, P.src[j], P.lt[j], coef + (size_t)mbi * kCoefStride, x * 16, y0,
                                    mb_avail(g, x, mby, slice_rows), e2);
                sse_a += e2;
                if (j == 0 ? um[0] : (j == 1 ? um[1] : um[2])) sse_m += e2;
                if (r == 0) mbs[mbi].nz_luma[rb] = (uint8_t)nzb;
            }
            const unsigned long long any = __ballot(rb >= 0 && r == 0 && nzb > 0);
            wave_sync_lds();
            // per slot (uniform): coded-block bits, right-column hand-off, completion
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                const int ks = sk[s], ss = t - 4 * ks;
                if (ks < 0 || ss > 9) continue;
#pragma unroll
                for (int gq = 0; gq < 2; ++gq)
                    if ((any >> (8 * s + 4 * gq)) & 1ull) cbp[s] |= 1 << (raster_to_blk(i4_step_block(ss, gq)) >> 2);
                if (ss >= 3 && (ss & 1)) {  // block (3, by) done: successor's left column rows 4by .. 4by+3
                    const int by = (ss - 3) >> 1, jn = s == 2 ? 0 : s + 1;  // slot of MB base + ks + 1
                    if (lane < 4) P.lt[jn][1 + 4 * by + lane][0] = P.lt[s][1 + 4 * by + lane][16];
                }
                if (ss == 9) {
                    if (lane == 0) mbs[mby * g.mb_w + base + ks].cbp = (uint8_t)cbp[s];
                    finish(base + ks);
                }
            }
            wave_sync_lds();
        }
        next = base + started;
    }
#ifdef MX_IDR_TIMING
    if (lane == 0) printf("MXIDR plane 0 slice %d row %d wall_ticks %llu\n", (int)blockIdx.x, wave, wall_clock64() - t_start);
#endif
    unsigned long long a = sse_a, mm = sse_m;
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        mm += __shfl_xor(mm, o, 64);
    }
    if (lane == 0) {
        fs->sse_part[0 * kSsePartStride + mby] = a;
        fs->sse_part[3 * kSsePartStride + mby] = mm;
    }
}

__global__ __launch_bounds__(512) void k_intra_wave(Geometry g, const FrameState* __restrict__ fs,
                                                     const uint8_t* __restrict__ src_y,
                                                     const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs,
                                                     int16_t* __restrict__ coef) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    extern __shared__ uint8_t s_line[];  // [slice rows][coded_w]: bottom sample line of every coded MB
    __shared__ IntraWaveTiles tiles[8];     // chroma workgroups
    __shared__ LumaPipeTiles ltiles[8];     // luma workgroups
    __shared__ int prog[8];              // macroblocks of the row whose bottom line is in s_line
    if ((threadIdx.x & 63) == 0) prog[threadIdx.x >> 6] = 0;
    __syncthreads();
    if (blockIdx.y == 0)
        intra_luma_rows_pl(g, fs, src_y, mbs, coef, s_line, ltiles, prog);
    else
        intra_wave_rows<true>(g, fs, src_y, src_uv, mbs, coef, s_line, tiles, prog);
}

// IDR: luma and chroma coded bits merged into the MB's cbp once both planes are done.
__global__ __launch_bounds__(256) void k_intra_cbp(Geometry g, MbInfo* __restrict__ mbs) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= g.mb_w * g.mb_h) return;
    MbInfo& m = mbs[i];
    m.cbp = (uint8_t)((m.cbp & 15) | (m.cbp_c << 4));
}

// Intra macroblocks of P pictures (independent by construction, see intra_selected()): one
// workgroup per macroblock, luma on wave 0 and chroma on wave 1, neighbours straight from the
// final inter reconstruction, coded by the same routines as k_intra_wave.  The distortion
// delta against the MB's inter distortion goes into its row's partial (atomic, few MBs).
__device__ void intra_p_mb(const Geometry& g, const FrameState* __restrict__ fs, const uint8_t* __restrict__ src_y,
                           const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs, int16_t* __restrict__ coef,
                           const int32_t* __restrict__ gain, const uint32_t* __restrict__ mb_sse, int mbi) {
    __shared__ uint8_t lt[17][kLT];
    __shared__ uint8_t ct[2][9][kCT];
    __shared__ uint32_t ls[64];
    __shared__ uint32_t cs[32];
    __shared__ int ldc[16], cdc[8];
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    if (!intra_selected(gain, g.mb_w, g.mb_h, mbx, mby)) return;  // uniform over the workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    MbInfo& m = mbs[mbi];
    MbFields f = load_fields(&m);
    f.type = m.itype;
    f.qp = fs->qp;
    const Avail av = mb_avail(g, mbx, mby, fs->slice_rows);
    int16_t* mc = coef + (size_t)mbi * kCoefStride;
    uint32_t s0 = 0, s1 = 0;
    __syncthreads();  // every wave has read the MB fields before they are overwritten
    if (threadIdx.x == 0) {
        m.type = (uint8_t)f.type;
        m.qp = (uint8_t)f.qp;
        m.mvx = 0;
        m.mvy = 0;
    }
    if (wave == 0) {
        const int x0 = mbx * 16, y0 = mby * 16;
        {
            const int r = lane >> 2, c4 = (lane & 3) * 4;
            ls[lane] = *reinterpret_cast<const uint32_t*>(src_y + (size_t)(y0 + r) * g.pitch + x0 + c4);
        }
        if (lane < 16) lt[1 + lane][0] = av.left ? fs->rec_y[(y0 + lane) * g.pitch + x0 - 1] : 0;
        if (lane < 21) {
            const bool ok = lane == 0 ? av.topleft : (lane <= 16 ? av.top : av.topright);
            lt[0][lane] = ok ? fs->rec_y[(y0 - 1) * g.pitch + x0 - 1 + lane] : 0;
        }
        wave_sync_lds();
        intra_luma_mb(g, f, ls, m, mc, mbx, mby, av, lt, ldc, lane, s0);
        const int r = lane >> 2, c4 = (lane & 3) * 4;
        const uint32_t v = (uint32_t)lt[1 + r][1 + c4] | ((uint32_t)lt[1 + r][2 + c4] << 8) |
                           ((uint32_t)lt[1 + r][3 + c4] << 16) | ((uint32_t)lt[1 + r][4 + c4] << 24);
        *reinterpret_cast<uint32_t*>(fs->rec_y + (y0 + r) * g.pitch + x0 + c4) = v;
    } else {
        const int xc0 = mbx * 8, yc0 = mby * 8;
        if (lane < 32) {
            const int r = lane >> 2, c4 = (lane & 3) * 4;
            cs[lane] = *reinterpret_cast<const uint32_t*>(src_uv + (size_t)(yc0 + r) * g.pitch + mbx * 16 + c4);
        }
        if (lane < 16) {
            const int comp = lane >> 3, r = lane & 7;
            ct[comp][1 + r][0] = av.left ? fs->rec_uv[(yc0 + r) * g.pitch + 2 * (xc0 - 1) + comp] : 0;
        } else if (lane < 34) {
            const int k = lane - 16, comp = k / 9, cx = k - comp * 9;
            const bool ok = cx == 0 ? av.topleft : av.top;
            ct[comp][0][cx] = ok ? fs->rec_uv[(yc0 - 1) * g.pitch + 2 * (xc0 - 1 + cx) + comp] : 0;
        }
        wave_sync_lds();
        intra_chroma_mb(g, fs->chroma_qp_offset, f, cs, m, mc, mbx, mby, av, ct, cdc, lane, s0, s1);
        if (lane < 32) {
            const int r = lane >> 2, c2 = (lane & 3) * 2;
            const uint32_t v = (uint32_t)ct[0][1 + r][1 + c2] | ((uint32_t)ct[1][1 + r][1 + c2] << 8) |
                               ((uint32_t)ct[0][1 + r][2 + c2] << 16) | ((uint32_t)ct[1][1 + r][2 + c2] << 24);
            *reinterpret_cast<uint32_t*>(fs->rec_uv + (yc0 + r) * g.pitch + 2 * (xc0 + c2)) = v;
        }
    }
    unsigned long long a = s0, b = s1;
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    __syncthreads();  // both waves done: merge the chroma cbp
    const int nmb = g.mb_w * g.mb_h;
    const int slot = (nmb + 3) / 4 + mby;
    if (lane == 0) {
        if (wave == 0) {
            m.cbp = (uint8_t)((m.cbp & 15) | (m.cbp_c << 4));
            atomicAdd(&fs->sse_part[slot], a - mb_sse[mbi]);
            if (mb_unmasked(fs, mbx, mby)) atomicAdd(&fs->sse_part[3 * kSsePartStride + slot], a - mb_sse[mbi]);
        } else {
            atomicAdd(&fs->sse_part[kSsePartStride + slot], a - mb_sse[nmb + mbi]);
            atomicAdd(&fs->sse_part[2 * kSsePartStride + slot], b - mb_sse[2 * nmb + mbi]);
        }
    }
}

__global__ __launch_bounds__(128) void k_intra_p(Geometry g, const FrameState* __restrict__ fs,
                                                 const uint8_t* __restrict__ src_y, const uint8_t* __restrict__ src_uv,
                                                 MbInfo* __restrict__ mbs, int16_t* __restrict__ coef,
                                                 const int32_t* __restrict__ gain, const uint32_t* __restrict__ mb_sse,
                                                 const int* __restrict__ wave_prog, const int* __restrict__ cand) {
    // the candidates (positive gain) listed by k_intra_analyze; a fixed grid walks the list
    const int ncand = wave_prog[1];
    for (int k = blockIdx.x; k < ncand; k += gridDim.x) intra_p_mb(g, fs, src_y, src_uv, mbs, coef, gain, mb_sse, cand[k]);
}

// ------------------------------------------------------------------ CAVLC
__device__ __forceinline__ uint32_t mask_bits(int n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1); }

// OR the overlap of segment [s0, s0+len) with output word [W0, W0+32) into acc; getbits
// returns `n` segment-relative bits starting at `a`.
template <class F>
__device__ __forceinline__ void overlap(uint32_t& acc, uint32_t W0, uint32_t s0, uint32_t len, F getbits) {
    const uint32_t lo = max(W0, s0), hi = min(W0 + 32, s0 + len);
    if (lo >= hi) return;
    const int n = (int)(hi - lo);
    const uint32_t bits = getbits(lo - s0, n) & mask_bits(n);
    acc |= bits << (W0 + 32 - hi);
}

// One wave per MB, one CAVLC "role" per lane.  Single coding pass: each role writes its bits
// MSB-first into a private LDS buffer; a wave prefix sum of the bit counts places the roles;
// then each lane assembles whole output words of the MB slot from the (at most a few) role
// buffers overlapping them and stores them straight to the global slot.
constexpr int kRoleWords = 24;  // worst-case CAVLC 4x4 block ~630 bits
__device__ __forceinline__ uint32_t role_get(const uint32_t* buf, uint32_t b, int n) {
    const uint32_t wi = b >> 5, sh = b & 31;
    const uint64_t hi = ((uint64_t)buf[wi] << 32) | (wi + 1 < (uint32_t)kRoleWords ? buf[wi + 1] : 0u);
    return (uint32_t)((hi << sh) >> (64 - n));
}

// Two macroblocks per wave (one per 32-lane half): the 28 roles of an MB fill a half, so a
// wave no longer idles 36 of its 64 lanes; the prefix sum, ballots and word assembly are
// segmented per half.
constexpr int kCavlcMbPerBlock = 8;
__global__ __launch_bounds__(256) void k_cavlc(Geometry g, const FrameState* __restrict__ fs, MbInfo* __restrict__ mbs,
                                               const int16_t* __restrict__ coef, uint32_t* __restrict__ slot,
                                               uint32_t* __restrict__ slot_bits) {
    static_assert(kNumRoles < 32, "the roles of one MB (plus the total slot) must fit a half-wave");
    __shared__ uint32_t rbuf[kCavlcMbPerBlock][kNumRoles][kRoleWords];
    __shared__ uint32_t roff[kCavlcMbPerBlock][kNumRoles + 1];
    __shared__ __attribute__((aligned(16))) int16_t cbuf[kCavlcMbPerBlock][kCoefStride];
    __shared__ MbInfo nbuf[kCavlcMbPerBlock][5];  // self, left, top, top-right, top-left
    static_assert(sizeof(MbInfo) % 4 == 0, "MbInfo copied as dwords");
    const int hw = (threadIdx.x >> 5) & 1, lane = threadIdx.x & 31;  // hw: half of the wave; lane = role
    const int wave = threadIdx.x >> 5;                                   // MB slot in the block (half-wave)
    const int nmb = g.mb_w * g.mb_h;
    const int mbi = blockIdx.x * kCavlcMbPerBlock + wave;
    if (mbi >= nmb) return;  // a whole half exits; only half-local shuffles below, no workgroup barrier
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    const Avail av = mb_avail(g, mbx, mby, fs->slice_rows);
    // the MB's and its available neighbours' MbInfo into LDS (12 dwords each, one load round):
    // the role coders read their fields in data-dependent order, from global memory that was
    // a chain of L2 round trips
    {
        const int src[5] = {mbi, mbi - 1, mbi - g.mb_w, mbi - g.mb_w + 1, mbi - g.mb_w - 1};
        const bool ok[5] = {true, av.left, av.top, av.topright, av.topleft};
        constexpr int kW = (int)(sizeof(MbInfo) / 4);
        for (int q = lane; q < 5 * kW; q += 32) {
            const int k = q / kW, d = q - k * kW;
            if (ok[k]) reinterpret_cast<uint32_t*>(&nbuf[wave][k])[d] = reinterpret_cast<const uint32_t*>(&mbs[src[k]])[d];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const MbNbrs nb{&nbuf[wave][0], &nbuf[wave][1], &nbuf[wave][2], &nbuf[wave][3], &nbuf[wave][4]};
    const MbInfo& m = nbuf[wave][0];
    const int16_t* mc = coef + (size_t)mbi * kCoefStride;

    // motion vector prediction + P_Skip decision (every lane computes the same values)
    int mvd[4];
    const bool skip = decide_skip(nb, av, mvd);
    // mb_qp_delta: QP predictor = QP of the previous MB in the slice that carried one (a P
    // macroblock with residual); skipped / residual-free MBs inherit it.  Half-wave-parallel
    // backward search (the ballot holds active lanes only; this half's bits are taken), 512 MBs
    // per step: each lane tests 16 (independent loads, one latency per step) -- static desktop
    // areas are long skip runs, and at 128 MBs per step the dependent steps through them were
    // ~7 us of k_cavlc (a separate scan kernel cost more than it saved: profiles/r03_h264).
    // I slices: every MB is at the slice QP.
    int dqp = 0;
    if (!skip && !fs->idr && carries_dqp(m)) {
        const int per_slice = fs->slice_rows * g.mb_w, first = (mbi / per_slice) * per_slice;
        int pred = fs->qp;
        bool found = false;
        constexpr int kPer = 16;
        for (int j0 = mbi - 1; j0 >= first && !found; j0 -= 32 * kPer) {
            int qv[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const int j = j0 - 32 * k - lane;
                qv[k] = -1;
                if (j >= first) {
                    const MbInfo& mj = mbs[j];
                    if (carries_dqp(mj)) qv[k] = mj.qp;
                }
            }
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const unsigned long long bal = __ballot(qv[k] >= 0);
                const uint32_t hb = (uint32_t)(bal >> (32 * hw));
                const int q = __shfl(qv[k], hb ? (int)(__ffs(hb) - 1) : 0, 32);
                if (!found && hb) {
                    pred = q;
                    found = true;
                }
            }
        }
        dqp = qp_delta(m.qp, pred);
    }
    // the MB's coefficients into LDS first (one 16-byte load per lane and pass): the CAVLC
    // scans re-read them in data-dependent loops, which from global memory were chains of
    // dependent L2 round trips
    if (!skip) {
        const uint4* src = reinterpret_cast<const uint4*>(mc);
        uint4* dst = reinterpret_cast<uint4*>(cbuf[wave]);
        for (int q = lane; q < kCoefStride / 8; q += 32) dst[q] = src[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t bits = 0;
    if (!skip && lane < kNumRoles) {
        BitWriter w;
        w.init(rbuf[wave][lane]);
        code_role(w, lane, g, fs->idr, nb, cbuf[wave], av, mvd, dqp);
        w.flush();
        bits = w.bits;
    }
    // exclusive prefix sum of bits over the half's lanes -> role offsets in the MB slot
    // (DPP: shift-add scan within rows of 16, then row_bcast:15 into the odd rows -- rows 0-1 and
    // 2-3 are the two halves -- instead of five lane-shuffle round trips)
    uint32_t incl = bits;
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xF, 0xF, false);  // row_shr:1
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xF, 0xF, false);  // row_shr:2
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xF, 0xF, false);  // row_shr:4
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x118, 0xF, 0xF, false);  // row_shr:8
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x142, 0xA, 0xF, false);  // row_bcast:15
    const uint32_t total = __shfl(incl, 31, 32);
    if (lane < kNumRoles) roff[wave][lane] = incl - bits;
    if (lane == kNumRoles) roff[wave][kNumRoles] = total;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool fits = total <= kSlotWords * 32u;
    if (!skip && fits) {
        const uint32_t nwords = (total + 31) >> 5;
        uint32_t* dst = slot + (size_t)mbi * kSlotWords;
        for (uint32_t wi = lane; wi < nwords; wi += 32) {
            const uint32_t W0 = wi * 32;
            // first role ending after W0 (roles are contiguous and in lane order)
            int r = 0;
            while (r < kNumRoles - 1 && roff[wave][r + 1] <= W0) ++r;
            uint32_t acc = 0;
            for (; r < kNumRoles; ++r) {
                const uint32_t o = roff[wave][r], len = roff[wave][r + 1] - o;
                if (o >= W0 + 32) break;
                if (len == 0) continue;
                overlap(acc, W0, o, len, [&](uint32_t x, int n) { return role_get(rbuf[wave][r], x, n); });
            }
            dst[wi] = acc;
        }
    }
    if (lane == 0) {
        slot_bits[mbi] = skip ? 0u : (fits ? total : 0xffffffffu);
        mbs[mbi].skip = skip ? 1 : 0;
    }
}

// ------------------------------------------------------------------ scan (two passes, one workgroup per MB row)
// The bitstream layout needs, for every coded MB, its unit's absolute bit offset: unit bits =
// ue(skip run) + MB bits, slices byte-aligned behind their headers.  Pass 1 (k_scan_rows)
// summarises each MB row; pass 2 (k_scan_out) has every workgroup rebuild the row / slice
// prefixes from those summaries (a few hundred values) and lay out its own row.  Both passes
// spread the work over mb_h workgroups (a single-workgroup scan was latency bound at ~25 us).
constexpr int kScanThreads = 256;
constexpr int kScanRowPer = 2;   // MBs per thread in a row: mb_w <= 512
constexpr int kScanMaxRows = 512;

template <typename T, typename Op>
__device__ __forceinline__ T blk_excl_scan(T v, T init, Op op, T* wbuf, T* total) {
    constexpr int kW = kScanThreads / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const T t = __shfl_up(incl, o, 64);
        if (lane >= o) incl = op(incl, t);
    }
    T excl = __shfl_up(incl, 1, 64);
    if (lane == 0) excl = init;
    if (lane == 63) wbuf[w] = incl;
    __syncthreads();
    T before = init, all = init;
    for (int k = 0; k < kW; ++k) {
        if (k < w) before = op(before, wbuf[k]);
        all = op(all, wbuf[k]);
    }
    __syncthreads();
    *total = all;
    return op(before, excl);
}

__device__ __forceinline__ uint32_t blk_excl_sum(uint32_t v, uint32_t* wbuf, uint32_t* total) {
    return blk_excl_scan<uint32_t>(v, 0u, [](uint32_t a, uint32_t b) { return a + b; }, wbuf, total);
}
__device__ __forceinline__ int blk_excl_max(int v, int init, int* wbuf, int* total) {
    return blk_excl_scan<int>(v, init, [](int a, int b) { return max(a, b); }, wbuf, total);
}

__device__ __forceinline__ SliceParams slice_params(const FrameState* fs, int s, int mb_w) {
    return make_slice_params(s * fs->slice_rows * mb_w, fs->idr, fs->frame_num, fs->log2_max_frame_num,
                             fs->idr_pic_id, fs->qp - fs->pic_init_qp, fs->deblock_off);
}

// Pass 1, row r: {first coded MB or -1, last coded MB or -1, coded count | overflow << 31,
// unit bits of the row excluding the skip-run prefix of its first coded MB (that run depends
// on earlier rows)}; and this row's share of the distortion partials.
// slot_bits[i]: 0 = P_Skip, 0xffffffff = slot overflow, else coded MB bits (>= 1).
__global__ __launch_bounds__(kScanThreads) void k_scan_rows(Geometry g, const FrameState* __restrict__ fs,
                                                            const uint32_t* __restrict__ slot_bits,
                                                            uint4* __restrict__ row_agg,
                                                            unsigned long long* __restrict__ row_sse,
                                                            const MbInfo* __restrict__ mbs, uint32_t* __restrict__ db_cnt) {
    __shared__ int wi[kScanThreads / 64];
    __shared__ uint32_t wu[kScanThreads / 64];
    const int t = threadIdx.x, r = blockIdx.x, base = r * g.mb_w;
    const bool idr = fs->idr != 0;
    // distortion partials of this row's share (one per intra MB row or per 4-MB inter workgroup,
    // plus the per-row intra deltas of k_intra_wave / k_intra_p; one per MB row from k_db_sse
    // when the in-loop filter is on)
    const int nmb = g.mb_w * g.mb_h;
    const int nparts = (idr || !fs->deblock_off) ? g.mb_h : (nmb + 3) / 4 + (fs->intra_in_p ? g.mb_h : 0);
    const int p0 = (int)((long long)nparts * r / g.mb_h), p1 = (int)((long long)nparts * (r + 1) / g.mb_h);
    unsigned long long acc[4] = {0, 0, 0, 0};
    for (int i = p0 + t; i < p1; i += kScanThreads)
        for (int c = 0; c < 4; ++c) acc[c] += fs->sse_part[c * kSsePartStride + i];
    uint32_t b[kScanRowPer];
    int last = -1, first = 0x7fffffff;
    uint32_t ncoded = 0, over = 0;
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        const int j = t * kScanRowPer + k;
        b[k] = j < g.mb_w ? slot_bits[base + j] : 0u;
        if (b[k] == 0xffffffffu) {
            over = 1;
            b[k] = 1;
        }
        if (b[k]) {
            last = base + j;
            first = min(first, base + j);
            ++ncoded;
        }
    }
    int lastall;
    int prev = blk_excl_max(last, -1, wi, &lastall);  // last coded MB of the row before this thread
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        if (!b[k]) continue;
        const int i = base + t * kScanRowPer + k;
        if (prev >= 0 && !idr) bits += (uint32_t)ue_len((uint32_t)(i - prev - 1));
        bits += b[k];
        prev = i;
    }
    uint32_t tb, tc, to;
    (void)blk_excl_sum(bits, wu, &tb);
    (void)blk_excl_sum(ncoded, wu, &tc);
    (void)blk_excl_sum(over, wu, &to);
    int firstall;
    (void)blk_excl_scan<int>(first, 0x7fffffff, [](int x, int y) { return min(x, y); }, wi, &firstall);
    if (t == 0)
        row_agg[r] = make_uint4((uint32_t)(lastall >= 0 ? firstall : -1), (uint32_t)lastall,
                                tc | (to ? 0x80000000u : 0u), tb);
    __shared__ unsigned long long red[4][kScanThreads / 64];
    for (int c = 0; c < 4; ++c) {
        unsigned long long v = acc[c];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((t & 63) == 0) red[c][t >> 6] = v;
    }
    __syncthreads();
    if (t < 4) {
        unsigned long long v = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) v += red[t][w];
        row_sse[t * kScanMaxRows + r] = v;
    }
    if (idr || !db_cnt) return;
    // adaptive in-loop filter: this row's temporal-class counts (h264_deblock.h db_auto_count)
    DbAutoCounts ac;
    for (int j = t; j < g.mb_w; j += kScanThreads) db_auto_count(mbs, g.mb_w, base + j, ac);
    uint32_t cv[3] = {ac.coherent, ac.changed, ac.moving};
    __shared__ uint32_t cred[3][kScanThreads / 64];
    for (int c = 0; c < 3; ++c) {
        for (int o = 32; o > 0; o >>= 1) cv[c] += __shfl_xor(cv[c], o);
        if ((t & 63) == 0) cred[c][t >> 6] = cv[c];
    }
    __syncthreads();
    if (t < 3) {
        uint32_t v = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) v += cred[t][w];
        if (v) atomicAdd(&db_cnt[t], v);
    }
}

// Pass 2, row r: row / slice prefixes from all rows' summaries, then this row's units:
// coded_info[rank] = {absolute bit offset, MB index, unit bits, skip run} and the quad -> unit
// table for k_pack (rank of the unit -- or of the slice's first / end unit for header /
// trailer bits -- holding each 128-bit output quad's first bit).  The workgroup of a slice's
// first row writes slice_info; row 0 writes the header and the frame distortion.
__global__ __launch_bounds__(kScanThreads) void k_scan_out(Geometry g, const FrameState* __restrict__ fs,
                                                           const uint32_t* __restrict__ slot_bits,
                                                           const uint4* __restrict__ row_agg,
                                                           const unsigned long long* __restrict__ row_sse,
                                                           uint4* __restrict__ coded_info,
                                                           uint32_t* __restrict__ slice_info, size_t out_bytes,
                                                           OutHeader* __restrict__ hdr,
                                                           uint32_t* __restrict__ quad_unit, uint32_t* __restrict__ db_cnt) {
    __shared__ int s_lbraw[kScanMaxRows + 1];    // last coded MB before row j (any slice), -1 = none
    __shared__ uint32_t s_P[kScanMaxRows + 1];   // unit bits before row j (frame-wide running sum)
    __shared__ uint32_t s_R[kScanMaxRows + 1];   // coded MBs before row j
    __shared__ uint32_t s_soff[kScanThreads + 1], s_sbytes[kScanThreads], s_hbits[kScanThreads];
    __shared__ int wi[kScanThreads / 64];
    __shared__ uint32_t wu[kScanThreads / 64];
    const int t = threadIdx.x, r = blockIdx.x, mb_w = g.mb_w, mb_h = g.mb_h;
    const bool idr = fs->idr != 0;
    const int srows = fs->slice_rows, ns = fs->num_slices;
    // this row's MB bits, loaded up front (independent of the prefix work below)
    const int base = r * mb_w;
    uint32_t b[kScanRowPer];
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        const int j = t * kScanRowPer + k;
        b[k] = j < mb_w ? slot_bits[base + j] : 0u;
    }
    // frame distortion (row 0): the per-row sums, reduced by the whole workgroup
    unsigned long long dsum[4] = {0, 0, 0, 0};
    if (r == 0)
        for (int j = t; j < mb_h; j += kScanThreads)
            for (int c = 0; c < 4; ++c) dsum[c] += row_sse[c * kScanMaxRows + j];
    // rows t*2, t*2+1 of the frame per thread (mb_h <= kScanMaxRows)
    uint4 ag[2];
    int lastr = -1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int j = 2 * t + k;
        ag[k] = j < mb_h ? row_agg[j] : make_uint4(0xffffffffu, 0xffffffffu, 0u, 0u);
        lastr = max(lastr, (int)ag[k].y);
    }
    int dummy, lastframe;
    int lb = blk_excl_max(lastr, -1, wi, &lastframe);
    uint32_t contrib[2], nc[2], over = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int j = 2 * t + k;
        contrib[k] = 0;
        nc[k] = ag[k].z & 0x7fffffffu;
        over |= ag[k].z >> 31;
        if (j < mb_h) {
            s_lbraw[j] = lb;
            const int sfirst = (j / srows) * srows * mb_w;
            const int pv = max(lb, sfirst - 1);
            contrib[k] = ag[k].w;
            if ((int)ag[k].x >= 0 && !idr) contrib[k] += (uint32_t)ue_len((uint32_t)((int)ag[k].x - pv - 1));
        }
        lb = max(lb, (int)ag[k].y);
    }
    uint32_t ptot, rtot, otot;
    uint32_t pex = blk_excl_sum(contrib[0] + contrib[1], wu, &ptot);
    uint32_t rex = blk_excl_sum(nc[0] + nc[1], wu, &rtot);
    (void)blk_excl_sum(over, wu, &otot);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int j = 2 * t + k;
        if (j < mb_h) {
            s_P[j] = pex;
            s_R[j] = rex;
        }
        pex += contrib[k];
        rex += nc[k];
    }
    if (t == 0) {
        s_P[mb_h] = ptot;
        s_R[mb_h] = rtot;
        s_lbraw[mb_h] = lastframe;
    }
    __syncthreads();
    // slice sizes (ns <= kScanThreads: IDR slices are >= mb_h / 16 rows, P pictures one slice)
    uint32_t sbytes = 0, hb = 0;
    if (t < ns) {
        const int fr = t * srows, er = min(fr + srows, mb_h);
        const int sfirst = fr * mb_w, slast = er * mb_w - 1;
        const uint32_t data = s_P[er] - s_P[fr];
        const int lastin = max(s_lbraw[er], sfirst - 1);
        const uint32_t trail = idr ? 0u : (uint32_t)(slast - lastin);
        BitCounter bc;
        bc.init(nullptr);
        write_slice_header(bc, slice_params(fs, t, mb_w));
        hb = bc.bits;
        const uint32_t bits = hb + data + (trail ? ue_len(trail) : 0) + 1;
        sbytes = (bits + 7) >> 3;
    }
    uint32_t total_bytes;
    const uint32_t soff = blk_excl_sum(sbytes, wu, &total_bytes);
    if (t < ns) {
        s_soff[t] = soff;
        s_sbytes[t] = sbytes;
        s_hbits[t] = hb;
    }
    __syncthreads();
    const uint32_t nquads_max = (uint32_t)((out_bytes + 15) / 16);
    auto mark_quads = [&](uint32_t a, uint32_t len, uint32_t rk) {  // quads starting in [a, a + len)
        if (len == 0) return;
        const uint32_t qe = min((a + len - 1) >> 7, nquads_max - 1);
        for (uint32_t q = (a + 127) >> 7; q <= qe; ++q) quad_unit[q] = rk;
    };
    const int s = r / srows, fr = s * srows, er = min(fr + srows, mb_h);
    const uint32_t sbase = s_soff[s] * 8 + s_hbits[s];  // output bit of the slice's first unit
    // slice-level records (the slice's first row)
    if (r == fr && t == 0) {
        const uint32_t data = s_P[er] - s_P[fr];
        const int sfirst = fr * mb_w, slast = er * mb_w - 1;
        const int lastin = max(s_lbraw[er], sfirst - 1);
        const uint32_t trail = idr ? 0u : (uint32_t)(slast - lastin);
        uint32_t* si = slice_info + kSliceInfo * s;
        si[0] = s_hbits[s];
        si[1] = s_soff[s];
        si[2] = s_sbytes[s];
        si[3] = trail;
        si[4] = sbase + data;  // data end (trailer start)
        si[5] = s_P[fr];
        si[6] = s_R[fr];  // coded MBs before the slice
        si[7] = s_R[er];
        if (total_bytes <= out_bytes) {  // header and trailer quads of the slice
            mark_quads(s_soff[s] * 8, s_hbits[s], s_R[fr]);
            const uint32_t dend = sbase + data;
            mark_quads(dend, s_soff[s] * 8 + s_sbytes[s] * 8 - dend, s_R[er]);
        }
    }
    if (r == 0) {
        __shared__ unsigned long long red[4][kScanThreads / 64];
        for (int c = 0; c < 4; ++c) {
            unsigned long long v = dsum[c];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if ((t & 63) == 0) red[c][t >> 6] = v;
        }
        __syncthreads();
        if (t < 4) {
            unsigned long long v = 0;
            for (int w = 0; w < kScanThreads / 64; ++w) v += red[t][w];
            if (t < 3)
                hdr->sse[t] = v;
            else
                hdr->sse_masked = v;
        }
        if (t == 0) {
            const bool over_b = total_bytes > out_bytes;
            hdr->total_bytes = over_b ? 0 : total_bytes;
            hdr->num_slices = ns;
            hdr->overflow = (otot ? 1u : 0u) | (over_b ? 2u : 0u);
            hdr->deblocked = fs->deblock_off ? 0u : 1u;
            hdr->db_coherent = db_cnt ? db_cnt[0] : 0u;
            hdr->db_changed = db_cnt ? db_cnt[1] : 0u;
            hdr->db_moving = db_cnt ? db_cnt[2] : 0u;
            if (db_cnt) db_cnt[0] = db_cnt[1] = db_cnt[2] = 0;  // re-armed for the slot's next frame
        }
    }
    // this row's units
    const int sfirst = fr * mb_w;
    int last = -1;
    uint32_t ncod = 0;
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        const int j = t * kScanRowPer + k;
        if (b[k] == 0xffffffffu) b[k] = 1;
        if (b[k]) {
            last = base + j;
            ++ncod;
        }
    }
    int prev = blk_excl_max(last, max(s_lbraw[r], sfirst - 1), wi, &dummy);
    uint32_t ub[kScanRowPer], run[kScanRowPer], ltot = 0;
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        ub[k] = 0;
        run[k] = 0;
        if (!b[k]) continue;
        const int i = base + t * kScanRowPer + k;
        run[k] = (uint32_t)(i - prev - 1);
        ub[k] = (idr ? 0u : (uint32_t)ue_len(run[k])) + b[k];
        ltot += ub[k];
        prev = i;
    }
    uint32_t rowbits, rowcoded;
    uint32_t off = sbase + (s_P[r] - s_P[fr]) + blk_excl_sum(ltot, wu, &rowbits);
    uint32_t rk = s_R[r] + blk_excl_sum(ncod, wu, &rowcoded);
#pragma unroll
    for (int k = 0; k < kScanRowPer; ++k) {
        if (!ub[k]) continue;
        const int i = base + t * kScanRowPer + k;
        coded_info[rk] = make_uint4(off, (uint32_t)i, ub[k], run[k]);
        mark_quads(off, ub[k], rk);
        off += ub[k];
        ++rk;
    }
}

// ------------------------------------------------------------------ pack (gather)
// n bits (1..32) starting at bit b of an MB slot.
__device__ __forceinline__ uint32_t slot_get(const uint32_t* slot, uint32_t b, int n) {
    const uint32_t wi = b >> 5, sh = b & 31;
    const uint64_t hi = ((uint64_t)slot[wi] << 32) | (wi + 1 < (uint32_t)kSlotWords ? slot[wi + 1] : 0u);
    return (uint32_t)((hi << sh) >> (64 - n));
}



// One thread per 32-bit output word, four lanes per 16-byte quad: each lane locates its
// word's first overlapping slice / MB unit (4-ary search over the dense per-rank unit
// records written by k_scan), assembles the word from the slice header / MB units / slice
// trailer bits that overlap it, and lane 0 of the quad gathers the four words with lane
// shuffles and writes them with one 16-byte store straight into pinned host memory.
// No atomics, no zero-fill pass, short dependent-load chains (latency-bound kernel).
__device__ void pack_body(const Geometry& g, const FrameState* __restrict__ fs, const uint32_t* __restrict__ slot,
                          const uint4* __restrict__ coded_info, const uint32_t* __restrict__ slice_info,
                          const OutHeader& h, uint8_t* __restrict__ host, const uint32_t* __restrict__ quad_unit);

__global__ __launch_bounds__(256) void k_pack(Geometry g, const FrameState* __restrict__ fs,
                                              const uint32_t* __restrict__ slot,
                                              const uint4* __restrict__ coded_info,
                                              const uint32_t* __restrict__ slice_info,
                                              const OutHeader* __restrict__ hdr, uint8_t* __restrict__ host,
                                              const uint32_t* __restrict__ quad_unit, uint32_t* __restrict__ done) {
    const OutHeader h = *hdr;
    pack_body(g, fs, slot, coded_info, slice_info, h, host, quad_unit);
    // the last workgroup to finish stamps the frame's end time into the host header (the host
    // reads it after the frame's completion event) and re-arms the counter for the next frame
    __syncthreads();
    if (threadIdx.x == 0) {
        // relaxed: only the count matters (the host reads the header after the frame's completion
        // event); acq_rel put an L2 write-back (buffer_wbl2) + invalidate around it in every one of
        // the workgroups
        const uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            reinterpret_cast<OutHeader*>(host)->t_end = wall_clock64();
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ void pack_body(const Geometry& g, const FrameState* __restrict__ fs, const uint32_t* __restrict__ slot,
                          const uint4* __restrict__ coded_info, const uint32_t* __restrict__ slice_info,
                          const OutHeader& h, uint8_t* __restrict__ host, const uint32_t* __restrict__ quad_unit) {
    const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    if (gid == 0) *reinterpret_cast<OutHeader*>(host) = h;
    uint32_t* hs = reinterpret_cast<uint32_t*>(host + sizeof(OutHeader));
    for (size_t s = gid; s < h.num_slices; s += stride) {
        hs[s] = slice_info[kSliceInfo * s + 1];
        hs[kMaxSlices + s] = slice_info[kSliceInfo * s + 2];
    }
    if (h.overflow) return;
    const bool idr = fs->idr != 0;
    const int ns = (int)h.num_slices;
    const uint32_t nquads = (h.total_bytes + 15) / 16;
    uint4* out = reinterpret_cast<uint4*>(host + kOutPayloadOffset);
    const int sub = threadIdx.x & 3;  // word within the quad
    // all four lanes of a quad iterate together (uniform trip count for the shuffles)
    for (size_t qbase = gid >> 2; qbase < ((nquads + 63) / 64) * 64; qbase += stride >> 2) {
        const bool active = qbase < nquads;
        uint32_t acc = 0;
        if (active) {
            const uint32_t W0 = (uint32_t)qbase * 128 + 32 * sub;
            const int qa = (int)quad_unit[qbase];  // unit holding the quad's first bit (k_scan)
            // last slice starting at or before W0
            int lo = 0, hi = ns - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (slice_info[kSliceInfo * mid + 1] * 8 <= W0) lo = mid; else hi = mid - 1;
            }
            for (int s = lo; s < ns; ++s) {
                const uint32_t sbit = slice_info[kSliceInfo * s + 1] * 8;
                if (sbit >= W0 + 32) break;
                const uint32_t hbits = slice_info[kSliceInfo * s + 0];
                const uint32_t dend = slice_info[kSliceInfo * s + 4];
                if (sbit + slice_info[kSliceInfo * s + 2] * 8 <= W0) continue;  // slice ends before the word
                const uint32_t trail = idr ? 0u : slice_info[kSliceInfo * s + 3];
                if (sbit + hbits > W0) {
                    uint32_t hw[4] = {0, 0, 0, 0};
                    BitWriter bw;
                    bw.init(hw);
                    write_slice_header(bw, slice_params(fs, s, g.mb_w));
                    bw.flush();
                    overlap(acc, W0, sbit, hbits, [&](uint32_t x, int n) { return slot_get(hw, x, n); });
                }
                if (dend > W0 && sbit + hbits < W0 + 32) {
                    // last coded unit of the slice starting at or before W0: from the quad's
                    // first unit, forward over the (at most a few) units inside the quad
                    int a = max((int)slice_info[kSliceInfo * s + 6], qa);
                    const int rend = (int)slice_info[kSliceInfo * s + 7];
                    const int b = rend - 1;
                    while (a < b && coded_info[a + 1].x <= W0) ++a;
                    for (int r = a; r < rend; ++r) {
                        const uint4 ci = coded_info[r];
                        const uint32_t off = ci.x;
                        if (off >= W0 + 32) break;
                        if (off + ci.z <= W0) continue;
                        const int run = (int)ci.w;
                        const int plen = idr ? 0 : ue_len((uint32_t)run);
                        const uint32_t pv = (uint32_t)run + 1;
                        const uint32_t* sp = slot + (size_t)ci.y * kSlotWords;
                        overlap(acc, W0, off, ci.z, [&](uint32_t x, int n) {
                            uint32_t r2 = 0;
                            int rem = n;
                            if ((int)x < plen) {
                                const int kk = min(rem, plen - (int)x);
                                r2 = (pv >> (plen - (int)x - kk)) & mask_bits(kk);
                                rem -= kk;
                                x += kk;
                            }
                            if (rem > 0) r2 = (rem == 32 ? 0u : (r2 << rem)) | slot_get(sp, x - plen, rem);
                            return r2;
                        });
                    }
                }
                const int tl = trail ? ue_len(trail) : 0;
                const uint32_t tv = trail ? (((trail + 1) << 1) | 1u) : 1u;
                overlap(acc, W0, dend, tl + 1, [&](uint32_t x, int n) { return tv >> (tl + 1 - (int)x - n); });
            }
        }
        const uint32_t w = bswap32(acc);
        const int lane = threadIdx.x & 63, q0 = lane & ~3;
        const uint32_t w0 = __shfl(w, q0), w1 = __shfl(w, q0 + 1), w2 = __shfl(w, q0 + 2), w3 = __shfl(w, q0 + 3);
        if (active && sub == 0) out[qbase] = make_uint4(w0, w1, w2, w3);
    }
}

}  // namespace

void launch_hpel(const Geometry& g, const DeviceBuffers& b, uint8_t* const planes[4], int hp_pitch,
                 hipStream_t stream, const FrameState* publish) {
    const int W = g.coded_w + 2 * kHpelPad, H = g.coded_h + 2 * kHpelPad;
    dim3 grid((W + kHpTW - 1) / kHpTW, (H + kHpTH - 1) / kHpTH);
    StateArg sa{};
    if (publish) sa.v = *publish;
    sa.dst = b.fs;
    sa.publish = publish ? 1 : 0;
    sa.t_start = b.out_hdr ? &b.out_hdr->t_start : nullptr;
    hipLaunchKernelGGL(k_hpel, grid, dim3(256), 0, stream, g, sa, planes[0], planes[1], planes[2], planes[3],
                       hp_pitch, (const uint8_t*)nullptr);
}

void launch_hpel_of(const Geometry& g, const uint8_t* luma, uint8_t* const planes[4], int hp_pitch, hipStream_t stream) {
    const int W = g.coded_w + 2 * kHpelPad, H = g.coded_h + 2 * kHpelPad;
    dim3 grid((W + kHpTW - 1) / kHpTW, (H + kHpTH - 1) / kHpTH);
    StateArg sa{};  // no state: the picture is given
    hipLaunchKernelGGL(k_hpel, grid, dim3(256), 0, stream, g, sa, planes[0], planes[1], planes[2], planes[3], hp_pitch,
                       luma);
}

void launch_me(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, hipStream_t stream,
               const FrameState* state) {
    const int nmb = g.mb_w * g.mb_h;
    if (state)
        hipLaunchKernelGGL(k_me_full_val, dim3(nmb), dim3(kMeThreads), 0, stream, g, *state, src_y, b.mb);
    else
        hipLaunchKernelGGL(k_me_full, dim3(nmb), dim3(kMeThreads), 0, stream, g, b.fs, src_y, b.mb);
}

void launch_inter(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream) {
    const int nmb = g.mb_w * g.mb_h;
    hipLaunchKernelGGL(k_inter_encode, dim3((nmb + 3) / 4), dim3(256), 0, stream, g, b.fs, src_y, src_uv, b.mb,
                       b.coef, b.mb_sse, b.wave_prog);
}

static void launch_analyze(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                           hipStream_t stream, const FrameState* publish, bool first) {
    const int nmb = g.mb_w * g.mb_h;
    StateArg sa{};
    if (publish) sa.v = *publish;
    sa.dst = b.fs;
    sa.publish = publish ? 1 : 0;
    // the first kernel of an I picture stamps the start; in a P picture k_hpel did
    sa.t_start = (b.out_hdr && first) ? &b.out_hdr->t_start : nullptr;
    hipLaunchKernelGGL(k_intra_analyze, dim3((nmb + 3) / 4), dim3(256), 0, stream, g, sa, src_y, src_uv, b.mb,
                       b.wave_prog, b.intra_gain, b.intra_cand);
}

void launch_intra_in_p(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                       hipStream_t stream) {
    launch_analyze(g, b, src_y, src_uv, stream, nullptr, false);
    // a fixed grid over k_intra_analyze's candidate list (a few percent of the MBs)
    hipLaunchKernelGGL(k_intra_p, dim3(256), dim3(128), 0, stream, g, b.fs, src_y, src_uv, b.mb, b.coef,
                       b.intra_gain, b.mb_sse, b.wave_prog, b.intra_cand);
}

void launch_intra(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream, const FrameState* publish) {
    launch_analyze(g, b, src_y, src_uv, stream, publish, true);
    // one workgroup per (slice, plane), one wave per slice row; LDS line buffers of the rows
    const int rows = idr_slice_rows(g.mb_h), slices = (g.mb_h + rows - 1) / rows;
    const size_t lds = (size_t)rows * g.coded_w;
    // line buffers above the default dynamic-LDS limit (8K: 61 KB + tiles); per device, once
    ensure_func_attr(reinterpret_cast<const void*>(&k_intra_wave), hipFuncAttributeMaxDynamicSharedMemorySize,
                     160 * 1024 - (int)(sizeof(IntraWaveTiles) + sizeof(LumaPipeTiles)) * 8 - 32);
    hipLaunchKernelGGL(k_intra_wave, dim3(slices, 2), dim3(64 * rows), lds, stream, g, b.fs, src_y, src_uv, b.mb,
                       b.coef);
    hipLaunchKernelGGL(k_intra_cbp, dim3((g.mb_w * g.mb_h + 255) / 256), dim3(256), 0, stream, g, b.mb);
}

__global__ __launch_bounds__(256) void k_save_src(Geometry g, const FrameState* __restrict__ fs,
                                                   const uint8_t* __restrict__ src_y) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // 16-byte chunk
    const size_t n = (size_t)g.pitch * g.coded_h / 16;
    if (i < n) reinterpret_cast<uint4*>(fs->save_src)[i] = reinterpret_cast<const uint4*>(src_y)[i];
}

void launch_save_src(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, hipStream_t stream) {
    const size_t n = (size_t)g.pitch * g.coded_h / 16;  // pitch is a multiple of 256
    hipLaunchKernelGGL(k_save_src, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, g, b.fs, src_y);
}

void launch_entropy(const Geometry& g, const DeviceBuffers& b, uint8_t* host_out, hipStream_t stream,
                    hipEvent_t wait_for_sse) {
    const int nmb = g.mb_w * g.mb_h;
    hipLaunchKernelGGL(k_cavlc, dim3((nmb + kCavlcMbPerBlock - 1) / kCavlcMbPerBlock), dim3(256), 0, stream, g, b.fs,
                       b.mb, b.coef, b.slot,
                       b.slot_bits);
    if (wait_for_sse) HIP_CHECK(hipStreamWaitEvent(stream, wait_for_sse, 0));
    if (g.mb_h > kScanMaxRows || g.mb_w > kScanThreads * kScanRowPer)
        throw std::runtime_error("launch_entropy: frame too large for the row scan");
    hipLaunchKernelGGL(k_scan_rows, dim3(g.mb_h), dim3(kScanThreads), 0, stream, g, b.fs, b.slot_bits, b.row_agg,
                       b.row_sse, b.mb, b.db_cnt);
    hipLaunchKernelGGL(k_scan_out, dim3(g.mb_h), dim3(kScanThreads), 0, stream, g, b.fs, b.slot_bits, b.row_agg,
                       b.row_sse, b.coded_info, b.slice_info, b.out_bytes, b.out_hdr, b.quad_unit, b.db_cnt);
    hipLaunchKernelGGL(k_pack, dim3(256), dim3(256), 0, stream, g, b.fs, b.slot, b.coded_info, b.slice_info,
                       b.out_hdr, host_out, b.quad_unit, b.pack_done);
}

}  // namespace h264
}  // namespace mx
