// H.264 in-loop deblocking filter on gfx950 (ITU-T H.264 8.7; shared arithmetic in h264_deblock.h).
//
// 8.7 filters macroblock by macroblock in raster order, and every macroblock reads samples its left
// neighbour's horizontal edges and its upper-right neighbour's left edge have already modified, so
// the filter is a wavefront.  It is mapped onto the hardware as follows:
//
//  * k_db_prep (one workgroup per MB row, fully parallel): every macroblock's boundary strengths
//    (4 edges x 4 segments x {vertical, horizontal}, 3 bits each) and its mb_qp_delta flag into a
//    16-byte record; per row, the QP of the last macroblock carrying mb_qp_delta (so a row can start
//    its running QP_Y without walking the picture).
//  * k_deblock: one wave per (MB row, plane) -- luma and chroma are independent -- walking its row
//    left to right; R = 4 rows per workgroup (one row wave per SIMD; the LDS is padded so no other
//    deblocking workgroup shares the CU) or 8 (MXDESK_DB_ROWS).  All edges of one direction of a
//    macroblock are filtered at once, one lane per (line, edge), and settled in 1-3 passes (the
//    luma engine's comment has the dependency argument); vertical edges run on row dwords in
//    registers (quad DPP moves carry the neighbouring edge's samples), horizontal edges on bytes
//    read back transposed from a per-wave LDS tile.  The step's control is scalar: the band's
//    boundary-strength records sit in VGPRs (lane j: MB xb + j) and are read with v_readlane, the
//    alpha / beta / tC0 and QP_C tables likewise (no memory access on the serial chain).  A row
//    hands each finished macroblock's bottom lines (luma rows 12..15, chroma rows 6..7: the p
//    samples of the next row's top edge) down through an LDS ring with a progress counter (the row
//    below waits only where its own top edge is filtered); the band's last row hands them to the
//    next workgroup (another XCD, another L2) through global memory as epoch-tagged 64-bit
//    agent-scope atomic words -- 32 sample bits and the frame's tag -- which the consumer polls
//    directly: no agent-scope release fence per macroblock (on gfx950 a write-back of the XCD's
//    whole L2).  Every sample byte has exactly one writer: rows 13..15 of a macroblock whose lower
//    neighbour filters its top edge are written by the row below, else by their own row.
//    Macroblocks with every bS == 0 (static desktop, skips with equal vectors) cost a record read
//    and a counter update, so P pictures pay for the changing areas only.  1080p pan (every MB
//    filtered): 332 -> ~220 us per picture against the earlier one-edge-at-a-time engine
//    (profiles/r06_deblock/NOTES.md).
//  * the distortion of the filtered picture (one partial per MB row and channel, replacing the
//    analysis kernels' unfiltered figures in the frame statistics) is summed by the row waves
//    themselves once their row is done, each over the samples it wrote (db_luma_sse): no separate
//    pass on the frame's chain (it was 25 us at 1080p).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

#include "../common/hip_check.h"
#include "h264_deblock.h"
#include "h264_gpu.h"
#include "h264_mb.h"

namespace mx {
namespace h264 {

namespace {

// MB rows (waves per plane) per workgroup: 8 (two row waves per SIMD) or 4 (one; the workgroup's
// LDS is padded past half the CU's so no other deblocking workgroup shares its SIMDs);
// MXDESK_DB_ROWS picks one at run time for measurement
constexpr int kDbRowsDefault = 4;
constexpr int kDbRing = 16;  // LDS hand-off slots per row
constexpr int kDbMaxW = 512; // MBs per row (the encoder's limit): the band's records live in LDS
constexpr int kDbPf = 8;     // macroblocks of sample lines prefetched ahead (one batch)
constexpr unsigned kDbSpinLimit = 1u << 22;
// global-memory words shared between workgroups: address-space-1 (global_*, never flat_*) atomics
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

// record word layout: w[dir * 2 + (e >> 1)] bits 12 * (e & 1) .. +11 = bS of edge e, segments 0..3
// (3 bits each); w[3] bits 24..29 = the MB's QP, bit 30 = carries mb_qp_delta
__device__ __forceinline__ uint32_t rec_edge(const uint4& r, int dir, int e) {
    const uint32_t w = dir == 0 ? (e < 2 ? r.x : r.y) : (e < 2 ? r.z : r.w);
    return (w >> (12 * (e & 1))) & 0xfffu;
}

__global__ __launch_bounds__(256) void k_db_prep(Geometry g, const FrameState* __restrict__ fs,
                                                 const MbInfo* __restrict__ mbs, uint4* __restrict__ rec,
                                                 int* __restrict__ row_lastq) {
    const int mby = blockIdx.x;
    __shared__ int best[4];
    int last = -1;  // (mbx << 8) | qp of the last dqp-carrying MB this thread saw
    for (int mbx = threadIdx.x; mbx < g.mb_w; mbx += 256) {
        const int i = mby * g.mb_w + mbx;
        const MbInfo q = mbs[i];
        MbInfo l, t;
        if (mbx > 0) l = mbs[i - 1];
        if (mby > 0) t = mbs[i - g.mb_w];
        uint32_t v[4], h[4];
        for (int e = 0; e < 4; ++e) {
            v[e] = db_edge_bs4(q, mbx > 0 ? &l : nullptr, e, true);
            h[e] = db_edge_bs4(q, mby > 0 ? &t : nullptr, e, false);
        }
        const bool dq = !fs->idr && carries_dqp(q);
        uint4 r;
        r.x = v[0] | (v[1] << 12);
        r.y = v[2] | (v[3] << 12);
        r.z = h[0] | (h[1] << 12);
        r.w = h[2] | (h[3] << 12) | ((uint32_t)(q.qp & 63) << 24) | (dq ? 1u << 30 : 0u);
        rec[i] = r;
        if (dq) last = (mbx << 8) | q.qp;
    }
    // row maximum of `last` (largest mbx wins)
    for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o, 64));
    if ((threadIdx.x & 63) == 0) best[threadIdx.x >> 6] = last;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int b = max(max(best[0], best[1]), max(best[2], best[3]));
        row_lastq[mby] = b < 0 ? -1 : (b & 0xff);
    }
}

template <int R>
struct DbShared {
    uint8_t lring[R][kDbRing][4][16];  // luma rows 12..15 of a finished MB
    uint8_t cring[R][kDbRing][2][16];  // chroma rows 6..7 (interleaved U/V)
    uint8_t ringq[2][R][kDbRing];      // the MB's QP_Y (per plane's own running value)
    int prog[2][R];                    // ring entries published (MB count)
    int cons[2][R];                    // MB steps finished by the row (for the row above's ring reuse)
    uint8_t tile[2 * R][20][16];       // per-wave transposition tile
    uint4 recs[R + 1][kDbMaxW];        // the band's records + the next row's (bS, QP)
    uint4 stage[2 * R][kDbPf][16];     // per-wave prefetched sample lines (lane-private slots)
    uint32_t params[52];                     // alpha | beta << 8 | packed tC0 << 13, by indexA
    uint8_t cqp[52];                         // QP_C of a clipped qP_I (Table 8-15)
    uint8_t pad[R == 4 ? 20480 : 4];         // R 4: > 80 KiB, one deblocking workgroup per CU
};
template <int R>
__device__ __forceinline__ int lds_cqp(const DbShared<R>& S, int qp, int offset) {
    const int q = qp + offset;
    return S.cqp[q < 0 ? 0 : (q > 51 ? 51 : q)];
}
template <int R>
__device__ __forceinline__ DbParams lds_params(const DbShared<R>& S, int qpav) {
    const uint32_t w = S.params[qpav < 0 ? 0 : (qpav > 51 ? 51 : qpav)];
    DbParams d;
    d.alpha = (int)(w & 0xff);
    d.beta = (int)((w >> 8) & 31);
    d.tc0 = w >> 13;
    return d;
}


__device__ __forceinline__ void lds_sync_wave() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS-only ordering: the ring hand-off never passes global data between waves of a workgroup, so
// the progress words need no global-memory drain (a workgroup-scope release waits vmcnt(0) every
// step, draining the prefetched lines and the pixel stores).
// LDS operations of a wave execute in order, so the producer only drains its own LDS writes
// (lgkmcnt) before the progress word and the consumer needs a compiler barrier after reading it.
__device__ __forceinline__ int lds_load(const int* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}
// publish an LDS progress value: the ring bytes written before it are visible to the reader
__device__ __forceinline__ void lds_store(int* p, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// publish an LDS progress value without draining: a wave's LDS operations are performed in issue
// order, so a reader that sees the value sees the ring bytes written before it (the compiler fence
// keeps the stores in that order)
__device__ __forceinline__ void lds_publish(int* p, int v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Filter parameters and chroma QP as scalar-memory tables (uniform index: s_load, no LDS round
// trip on the row's serial chain)
struct DbTabs {
    uint32_t par[52];  // alpha | beta << 8 | packed tC0 << 13, by indexA
    uint32_t cqp[52];  // QP_C of a clipped qP_I (Table 8-15)
};
constexpr DbTabs make_db_tabs() {
    DbTabs t{};
    for (int i = 0; i < 52; ++i) {
        t.par[i] = (uint32_t)kDbAlpha[i] | ((uint32_t)kDbBeta[i] << 8) |
                   (((uint32_t)kDbTc0[i][0] | ((uint32_t)kDbTc0[i][1] << 5) | ((uint32_t)kDbTc0[i][2] << 10)) << 13);
        t.cqp[i] = (uint32_t)kChromaQp[i];
    }
    return t;
}
__constant__ DbTabs c_db_tabs = make_db_tabs();
// The tables live in two VGPRs of every row wave (lane i: entry i), read with v_readlane: no
// memory access on the chain (a scalar load would also drain the wave's pending LDS reads, which
// share its lgkmcnt counter)
struct DbLaneTabs {
    uint32_t par, cqp;
};
__device__ __forceinline__ DbLaneTabs load_lane_tabs(int lane) {
    const int i = lane < 52 ? lane : 51;
    return DbLaneTabs{c_db_tabs.par[i], c_db_tabs.cqp[i]};
}
__device__ __forceinline__ DbParams spar(const DbLaneTabs& T, int qpav) {
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)T.par, qpav < 0 ? 0 : (qpav > 51 ? 51 : qpav));
    DbParams d;
    d.alpha = (int)(w & 0xff);
    d.beta = (int)((w >> 8) & 31);
    d.tc0 = w >> 13;
    return d;
}
__device__ __forceinline__ int scqp(const DbLaneTabs& T, int qp, int offset) {
    const int q = qp + offset;
    return __builtin_amdgcn_readlane((int)T.cqp, q < 0 ? 0 : (q > 51 ? 51 : q));
}
__device__ __forceinline__ uint4 rd_lane(const uint4& v, int j) {
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)v.x, j), (uint32_t)__builtin_amdgcn_readlane((int)v.y, j),
                      (uint32_t)__builtin_amdgcn_readlane((int)v.z, j), (uint32_t)__builtin_amdgcn_readlane((int)v.w, j));
}

// 16-byte global load / store through address-space-1 pointers of a native vector type (a generic
// access -- or one through HIP's uint4 class, whose copy constructor takes a generic reference --
// compiles to flat_*, which also counts on lgkmcnt and so stalls every later LDS wait)
typedef unsigned DbV4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) DbV4 GDbV4;
__device__ __forceinline__ uint4 gld16(const uint8_t* p) {
    const DbV4 v = *(const GDbV4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst16(uint8_t* p, const uint4& v) {
    const DbV4 d = {v.x, v.y, v.z, v.w};
    *(GDbV4*)p = d;
}

// bounded spin until *p >= need (LDS, same workgroup); false on timeout
__device__ __forceinline__ bool wait_lds(const int* p, int need, int* err) {
    for (unsigned s = 0; lds_load(p) < need; ++s) {
        if (s > kDbSpinLimit) {
            *err = 1;
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return true;
}
__device__ __forceinline__ void unpack16(const uint4& v, int* o) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xff;
}
__device__ __forceinline__ uint4 pack16(const int* o) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k >> 2] |= (uint32_t)(o[k] & 0xff) << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// QP_Y entering row `mby` (P pictures, one slice: the last dqp MB of an earlier row, else the slice QP)
__device__ __forceinline__ int row_entry_qp(const FrameState* fs, const int* row_lastq, int mby, int lane) {
    if (fs->idr) return fs->qp;
    for (int r0 = mby - 1; r0 >= 0; r0 -= 64) {
        const int r = r0 - lane;
        const int q = r >= 0 ? row_lastq[r] : -1;
        const unsigned long long bal = __ballot(q >= 0);
        if (bal) return __shfl(q, __ffsll((long long)bal) - 1, 64);
    }
    return fs->qp;
}

// Band-boundary hand-off words: [plane][mb_h][mb_w][kDbGlbWords], each 32 payload bits (luma rows
// 12..15 of the band's last row: words 0..15; chroma rows 6..7 interleaved: words 0..7; then the
// MB's QP_Y) with the frame's epoch tag above them -- the consumer polls the words themselves, so
// the producer needs no agent-scope release fence (a write-back of the XCD's L2) per macroblock.
constexpr int kDbGlbWords = 24;
constexpr int kDbQWord = 16;  // QP_Y word (luma; chroma uses word 8)
struct DbGlobal {
    uint64_t* glb;    // [2][mb_h][mb_w][kDbGlbWords] tagged hand-off words of band-last rows
    int* err;         // mapped host word: a bounded spin timed out
    const uint8_t* src_y;   // the picture's source (distortion of the filtered picture)
    const uint8_t* src_uv;
};
// poll tagged words (lanes with need) until every one carries `epoch`; returns this lane's payload
__device__ __forceinline__ uint32_t poll_tagged(const uint64_t* p, bool need, uint32_t epoch, int* err) {
    uint64_t w = 0;
    const gu64* wp = (const gu64*)p;
    for (unsigned s = 0;; ++s) {
        if (need) w = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!__any(need && (uint32_t)(w >> 32) != epoch)) break;
        if (s > kDbSpinLimit) {
            *err = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return (uint32_t)w;
}
__device__ __forceinline__ void put_tagged(uint64_t* p, uint32_t v, uint32_t epoch) {
    __hip_atomic_store((gu64*)p, (uint64_t)v | ((uint64_t)epoch << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Diagnostics: device wall-clock (start, end) of the last picture's row waves, [plane][mby][2], and
// the ticks each row wave spent waiting (ring slot free, row above's progress, band hand-off
// words) (read by deblock_row_stamps(); a few stores per wave per picture)
__device__ unsigned long long g_db_stamps[2][kMaxSlices][2];
__device__ unsigned long long g_db_clk[2][kMaxSlices];  // shader-clock cycles of each row wave
__device__ unsigned long long g_db_waits[2][kMaxSlices][3];
__device__ unsigned long long g_db_phase[kMaxSlices][4];  // luma: ticks in step head, V, final, H

// ---------------------------------------------------------------- luma row engine
// Edge-parallel form.  8.7 orders a macroblock's luma edges (vertical 0..3, then horizontal
// 0..3), but the data dependencies between consecutive edges of one direction are shallow: for
// the normal filter (bS < 4, every internal edge) q1' depends on p1, p0, q0, q1, q2 only -- never
// on p2 or p3, the two samples the previous edge may have written -- so an edge's outputs depend
// on its left (upper) neighbour edge only through p2 = that edge's q1' (and, behind a bS-4 MB
// edge, p1 = its q2').  All four edges of a direction are therefore computed at once, one lane
// per (line, edge) -- 16 lines x 4 edges = the whole wave -- and corrected by re-evaluating each
// edge with its neighbour's outputs: two passes settle every edge, a third one an edge 2 behind a
// strong (bS 4) edge 0.  Layouts: vertical edges, lane 4r + e holds row r, columns 4e..4e+3 (one
// dword); horizontal edges, lane 4c + e holds column c, rows 4e-4..4e+3 as bytes read from a
// per-wave LDS tile.  Quad DPP moves carry the neighbour values.
template <int kCtrl>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xf, 0xf, false);
}
constexpr int kQuadShr1 = 0x90;   // lane e of a quad reads quad lane max(e - 1, 0)
constexpr int kQuadShl1 = 0xF9;   // quad lane min(e + 1, 3)
constexpr int kQuadBcast0 = 0x00; // quad lane 0
constexpr int kQuadBcast3 = 0xFF; // quad lane 3
struct Px8 {
    int p3, p2, p1, p0, q0, q1, q2, q3;
};
__device__ __forceinline__ Px8 px8(uint32_t p, uint32_t q) {
    return Px8{(int)(p & 0xff), (int)((p >> 8) & 0xff), (int)((p >> 16) & 0xff), (int)(p >> 24),
               (int)(q & 0xff), (int)((q >> 8) & 0xff), (int)((q >> 16) & 0xff), (int)(q >> 24)};
}
__device__ __forceinline__ Px8 edge_eval(Px8 v, int bs, const DbParams& d) {
    db_luma_line(v.p3, v.p2, v.p1, v.p0, v.q0, v.q1, v.q2, v.q3, bs, d);
    return v;
}
// Settle the four edges of one direction (see above): `in` = the lane's samples before any edge
// of the direction, `passes` 1..3.  Lane e >= 1 re-reads its p3 / p2 / p1 from edge e - 1's
// q0' / q1' / q2' (quad lane e - 1) each pass.
__device__ __forceinline__ Px8 settle_edges(const Px8& in, int bs, const DbParams& d, int e, int passes) {
    Px8 o = edge_eval(in, bs, d);
    for (int k = 1; k < passes; ++k) {
        const uint32_t l = qperm<kQuadShr1>((uint32_t)o.q0 | ((uint32_t)o.q1 << 8) | ((uint32_t)o.q2 << 16));
        Px8 v = in;
        if (e >= 1) {
            v.p3 = (int)(l & 0xff);
            v.p2 = (int)((l >> 8) & 0xff);
            v.p1 = (int)((l >> 16) & 0xff);
        }
        o = edge_eval(v, bs, d);
    }
    return o;
}
// passes to settle a direction: 1 with only edge 0 filtered; 2 when an internal edge is (or edge 1
// must take up a strong edge 0's q2' as its p1); 3 when both (edge 2 behind edge 1's changed q1')
__device__ __forceinline__ int edge_passes(bool internal, bool strong0) {
    return 1 + ((internal || strong0) ? 1 : 0) + ((internal && strong0) ? 1 : 0);
}
__device__ __forceinline__ uint32_t pk4(int a, int b, int c, int d) {
    return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}
__device__ __forceinline__ DbParams sel_params(bool first, const DbParams& a, const DbParams& b) {
    DbParams d;
    d.alpha = first ? a.alpha : b.alpha;
    d.beta = first ? a.beta : b.beta;
    d.tc0 = first ? a.tc0 : b.tc0;
    return d;
}
typedef __attribute__((address_space(1))) uint32_t GDbU32;
__device__ __forceinline__ uint32_t gld4(const uint8_t* p) { return *(const GDbU32*)p; }
__device__ __forceinline__ void gst4(uint8_t* p, uint32_t v) { *(GDbU32*)p = v; }

template <int kCtrl>
__device__ __forceinline__ uint32_t dppmov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xf, 0xf, false);
}
constexpr int kRowShl2 = 0x102, kRowShl6 = 0x106, kRowShr2 = 0x112, kRowShr6 = 0x116;
constexpr int kQuadSwap1 = 0xB1;  // quad_perm [1,0,3,2]: the other component's lane
__device__ __forceinline__ uint32_t blend(uint32_t a, uint32_t b, bool take_a) {
    return b ^ ((a ^ b) & (take_a ? 0xffffffffu : 0u));
}

// Distortion of the filtered picture, accounted by each sample's writer once the writer's row is
// done (replaces a separate k_db_sse pass on the frame's chain): a row wave sums its own
// macroblocks' rows 0..12, and rows 13..15 where the row below leaves them, plus the upper row's
// rows 13..15 it wrote itself (its filtered top edges); every lane re-reads only dwords it wrote
// or that nobody in this kernel writes, so no cross-wave visibility is involved.  Partials:
// sse_part[c][mby] (Y, U, V, Y outside the quality mask), the layout k_scan_rows sums.
__device__ void db_luma_sse(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                            const uint8_t* __restrict__ src_y, int mby, int lane) {
    const int r = lane >> 2, e = lane & 3, mb_w = g.mb_w, pitch = g.pitch;
    const bool pic_last = mby == g.mb_h - 1;
    const uint8_t* Y = fs->rec_y;
    unsigned long long sy = 0, sm = 0;
    auto sse4 = [](uint32_t a, uint32_t b, int nvis) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (int)((a >> (8 * k)) & 0xff) - (int)((b >> (8 * k)) & 0xff);
            acc += k < nvis ? (uint32_t)(d * d) : 0u;
        }
        return acc;
    };
    for (int xb = 0; xb < mb_w; xb += 64) {
        const int xm = min(xb + lane, mb_w - 1);
        const uint32_t t0v = rec[(size_t)mby * mb_w + xm].z & 0xfffu;
        const uint32_t btv = pic_last ? 0u : (rec[(size_t)(mby + 1) * mb_w + xm].z & 0xfffu);
        const int xe = min(mb_w, xb + 64);
        for (int x = xb; x < xe; ++x) {
            const bool t0 = __builtin_amdgcn_readlane((int)t0v, x - xb) != 0;
            const bool below = __builtin_amdgcn_readlane((int)btv, x - xb) != 0;
            const int cx = 16 * x + 4 * e, nvis = min(4, max(0, g.width - cx));
            const int yy = mby * 16 + r;
            uint32_t acc = 0, accm = 0;
            if ((r <= 12 || !below) && yy < g.height) {
                const uint32_t a = gld4(src_y + (size_t)yy * pitch + cx), b = gld4(Y + (size_t)yy * pitch + cx);
                acc = sse4(a, b, nvis);
                if (mb_unmasked(fs, x, mby)) accm = acc;
            }
            if (t0 && r >= 1 && r < 4) {  // the upper macroblock's rows 13..15, written by this row
                const int ya = mby * 16 - 4 + r;
                const uint32_t a = gld4(src_y + (size_t)ya * pitch + cx), b = gld4(Y + (size_t)ya * pitch + cx);
                const uint32_t v = sse4(a, b, nvis);
                acc += v;
                if (mb_unmasked(fs, x, mby - 1)) accm += v;
            }
            sy += acc;
            sm += accm;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        sy += __shfl_xor(sy, o, 64);
        sm += __shfl_xor(sm, o, 64);
    }
    if (lane == 0) {
        fs->sse_part[0 * kSsePartStride + mby] = sy;
        fs->sse_part[3 * kSsePartStride + mby] = sm;
    }
}
// Chroma: rows 0..6 (and 7 where the row below leaves it) and the upper row's row 7 it wrote.
__device__ void db_chroma_sse(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                              const uint8_t* __restrict__ src_uv, int mby, int lane) {
    const int k = lane >> 3, dq4 = (lane >> 1) & 3, comp = lane & 1, mb_w = g.mb_w, pitch = g.pitch;
    const bool pic_last = mby == g.mb_h - 1;
    const uint8_t* UV = fs->rec_uv;
    unsigned long long su = 0, sv = 0;
    auto sse2 = [](uint32_t a, uint32_t b, int nvis, uint32_t* u, uint32_t* v) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int d = (int)((a >> (8 * kk)) & 0xff) - (int)((b >> (8 * kk)) & 0xff);
            const uint32_t e2 = kk < nvis ? (uint32_t)(d * d) : 0u;
            if (kk & 1) *v += e2; else *u += e2;
        }
    };
    for (int xb = 0; xb < mb_w; xb += 64) {
        const int xm = min(xb + lane, mb_w - 1);
        const uint32_t t0v = rec[(size_t)mby * mb_w + xm].z & 0xfffu;
        const uint32_t btv = pic_last ? 0u : (rec[(size_t)(mby + 1) * mb_w + xm].z & 0xfffu);
        const int xe = min(mb_w, xb + 64);
        for (int x = xb; x < xe; ++x) {
            const bool t0 = __builtin_amdgcn_readlane((int)t0v, x - xb) != 0;
            const bool below = __builtin_amdgcn_readlane((int)btv, x - xb) != 0;
            const int cx = 16 * x + 4 * dq4, nvis = min(4, max(0, g.width - cx));
            const int yy = mby * 8 + k;
            uint32_t u = 0, v = 0;
            if (comp == 0 && (k <= 6 || !below) && 2 * yy < g.height)
                sse2(gld4(src_uv + (size_t)yy * pitch + cx), gld4(UV + (size_t)yy * pitch + cx), nvis, &u, &v);
            if (t0 && lane < 4) {  // the upper macroblock's row 7: dword `lane`, as the H phase stored it
                const int ya = mby * 8 - 1, cxa = 16 * x + 4 * lane, nva = min(4, max(0, g.width - cxa));
                sse2(gld4(src_uv + (size_t)ya * pitch + cxa), gld4(UV + (size_t)ya * pitch + cxa), nva, &u, &v);
            }
            su += u;
            sv += v;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        su += __shfl_xor(su, o, 64);
        sv += __shfl_xor(sv, o, 64);
    }
    if (lane == 0) {
        fs->sse_part[1 * kSsePartStride + mby] = su;
        fs->sse_part[2 * kSsePartStride + mby] = sv;
    }
}

template <int R>
__device__ void db_luma_row(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                            const int* __restrict__ row_lastq, DbShared<R>& S, const DbGlobal& G, int band_row,
                            int mby, int lane) {
    unsigned long long w_cons = 0, w_prog = 0, w_glb = 0;  // diagnostics: ticks spent waiting
    uint8_t* Y = fs->rec_y;
    const int pitch = g.pitch, mb_w = g.mb_w;
    const uint32_t epoch = (uint32_t)fs->db_epoch;  // full 32-bit tag above the 32 payload bits
    const bool band_first = band_row == 0, band_last = band_row == R - 1 || mby == g.mb_h - 1;
    const bool pic_last = mby == g.mb_h - 1;
    const int r = lane >> 2, e = lane & 3;  // vertical layout: row r, columns 4e..; horizontal: column r, rows 4e-4..
    int* prog_me = &S.prog[0][band_row];
    int* cons_me = &S.cons[0][band_row];
    uint8_t(*tile)[16] = S.tile[band_row];
    const DbLaneTabs T = load_lane_tabs(lane);
    int qrun = __builtin_amdgcn_readfirstlane(row_entry_qp(fs, row_lastq, mby, lane));
    int qprev = qrun;
    uint32_t prev = 0;      // MB x-1, vertical layout, final after its horizontal edges (cols 13..15 aside)
    bool prev_mod = false;  // MB x-1 was modified (its own edges)
    // sample dwords: batches of kDbPf macroblocks loaded one batch ahead into registers and parked
    // in the wave's LDS stage; each step reads the next step's dword from the stage, so no LDS
    // latency sits at the head of a step
    uint32_t pf[kDbPf];
    uint32_t(*stage)[64] = reinterpret_cast<uint32_t(*)[64]>(S.stage[band_row]);
    const uint8_t* line = Y + (size_t)(mby * 16 + r) * pitch + 4 * e;
    auto issue = [&](int xb) {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j) pf[j] = gld4(line + 16 * min(xb + j, mb_w - 1));
    };
    auto park = [&]() {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j) stage[j][lane] = pf[j];
    };
    issue(0);
    park();
    issue(kDbPf);
    uint32_t cur_nx = stage[0][lane];
    // the band's records in registers, 64 macroblocks per batch (lane j: MB xb + j), read per step
    // with v_readlane: the step's control flow is scalar
    uint4 rb = make_uint4(0, 0, 0, 0);
    uint32_t rbt = 0;          // the row below's top-edge bS of the same macroblocks
    bool below_prev = false;   // the row below filters the top edge of MB x-1
    for (int x = 0; x <= mb_w; ++x) {
        const bool have = x < mb_w;
        if (have && (x & 63) == 0) {
            const int xm = min(x + lane, mb_w - 1);
            rb = S.recs[band_row][xm];
            rbt = pic_last ? 0u : (S.recs[band_row + 1][xm].z & 0xfffu);
        }
        uint4 rr = make_uint4(0, 0, 0, 0);
        bool below_cur = false;
        if (have) {
            rr = rd_lane(rb, x & 63);
            below_cur = __builtin_amdgcn_readlane((int)rbt, x & 63) != 0;
        }
        uint32_t cur = cur_nx;
        if ((x + 1) % kDbPf == 0) {
            park();
            issue(x + 1 + kDbPf);
        }
        cur_nx = stage[(x + 1) % kDbPf][lane];
        if (have && (rr.w >> 30) & 1) qrun = (rr.w >> 24) & 63;
        const int qp = qrun;
        const DbParams dq = spar(T, qp), dl = spar(T, (qprev + qp + 1) >> 1);
        // ---- vertical edges of MB x; edge 0 also finishes MB x-1's columns 13..15
        const bool vmod = have && (rr.x | rr.y) != 0, v0 = have && (rr.x & 0xfffu) != 0;
        if (vmod) {
            const uint32_t w = e < 2 ? rr.x : rr.y;
            const int bs = (int)((w >> (12 * (e & 1) + 3 * (r >> 2))) & 7u);
            // both moves on every lane, then a bitwise blend (blend()): a select of two DPP results lets
            // the compiler branch on it and run each move with only its own lanes enabled, so the
            // source lanes of the other side read as 0
            const uint32_t pw = blend(qperm<kQuadBcast3>(prev), qperm<kQuadShr1>(cur), e == 0);
            const bool internal = ((rr.x >> 12) | rr.y) != 0;
            const bool strong0 = __any(e == 0 && bs == 4);
            const Px8 o = settle_edges(px8(pw, cur), bs, sel_params(e == 0, dl, dq), e, edge_passes(internal, strong0));
            const uint32_t mine = pk4(o.q0, o.q1, o.q2, o.q3), pside = pk4(o.p3, o.p2, o.p1, o.p0);
            const uint32_t nxt = qperm<kQuadShl1>(pside), e0p = qperm<kQuadBcast0>(pside);
            cur = blend((mine & 0xffffu) | (nxt & 0xffff0000u), mine, e < 3);
            prev = blend(e0p, prev, e == 3 && v0);
        }
        // ---- MB x-1 is final (except rows 13..15 when the row below filters its top edge)
        if (x > 0) {
            const int xp = x - 1;
            const bool below_top = below_prev;
            if ((prev_mod || v0) && (r <= 12 || !below_top))
                gst4(Y + (size_t)(mby * 16 + r) * pitch + 16 * xp + 4 * e, prev);
            if (below_top) {
                if (!band_last) {
                    const int slot = xp % kDbRing;
                    { const unsigned long long t = wall_clock64(); wait_lds(&S.cons[0][band_row + 1], xp - kDbRing + 1, G.err); w_cons += wall_clock64() - t; }  // ring slot free
                    if (r >= 12) *reinterpret_cast<uint32_t*>(&S.lring[band_row][slot][r - 12][4 * e]) = prev;
                    if (lane == 0) S.ringq[0][band_row][slot] = (uint8_t)qprev;
                } else {
                    uint64_t* dst = G.glb + ((size_t)(0 * g.mb_h + mby) * mb_w + xp) * kDbGlbWords;
                    if (r >= 12) put_tagged(dst + lane - 48, prev, epoch);
                    if (lane == 0) put_tagged(dst + kDbQWord, (uint32_t)qprev, epoch);
                }
            }
            if (!band_last && lane == 0) lds_publish(prog_me, x);
        }
        if (!have) break;
        // ---- horizontal edges of MB x (columns: lane 4c + e reads rows 4e-4 .. 4e+3 of the tile)
        const uint32_t t0 = rec_edge(rr, 1, 0);
        const bool hmod = (rr.z | (rr.w & 0xffffffu)) != 0;
        if (hmod) {
            int qtop = qp;
            if (t0) {  // the row above's bottom lines of MB x -> tile rows 0..3
                if (!band_first) {
                    { const unsigned long long t = wall_clock64(); wait_lds(&S.prog[0][band_row - 1], x + 1, G.err); w_prog += wall_clock64() - t; }
                    const int slot = x % kDbRing;
                    if (lane < 16)
                        *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) =
                            *reinterpret_cast<const uint32_t*>(&S.lring[band_row - 1][slot][lane >> 2][4 * (lane & 3)]);
                    qtop = __builtin_amdgcn_readfirstlane(S.ringq[0][band_row - 1][slot]);
                } else {
                    // rows 12..15 of the band above (lanes 0..15, a word each) and its QP_Y (lane 16);
                    // the poll retires its loads here (a vmcnt(0) at the merge below otherwise)
                    const uint64_t* src = G.glb + ((size_t)(0 * g.mb_h + mby - 1) * mb_w + x) * kDbGlbWords;
                    const unsigned long long tq = wall_clock64();
                    const uint32_t v = poll_tagged(src + (lane <= kDbQWord ? lane : 0), lane <= kDbQWord, epoch, G.err);
                    w_glb += wall_clock64() - tq;
                    if (lane < 16) *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) = v;
                    qtop = __builtin_amdgcn_readlane((int)v, kDbQWord);
                }
            }
            *reinterpret_cast<uint32_t*>(&tile[4 + r][4 * e]) = cur;
            const DbParams dt = spar(T, (qtop + qp + 1) >> 1);
            lds_sync_wave();
            Px8 in;
            in.p3 = tile[4 * e][r];
            in.p2 = tile[4 * e + 1][r];
            in.p1 = tile[4 * e + 2][r];
            in.p0 = tile[4 * e + 3][r];
            in.q0 = tile[4 * e + 4][r];
            in.q1 = tile[4 * e + 5][r];
            in.q2 = tile[4 * e + 6][r];
            in.q3 = tile[4 * e + 7][r];
            const uint32_t w = e < 2 ? rr.z : rr.w;
            const int bs = (int)((w >> (12 * (e & 1) + 3 * (r >> 2))) & 7u);
            const bool internal = ((rr.z >> 12) | (rr.w & 0xffffffu)) != 0;
            const bool strong0 = __any(e == 0 && bs == 4);
            const Px8 o = settle_edges(in, bs, sel_params(e == 0, dt, dq), e, edge_passes(internal, strong0));
            lds_sync_wave();  // every lane's reads done before the tile is rewritten
            // Each lane writes rows no other lane writes (the compiler may reorder one lane's stores,
            // so lanes must not race on a byte): edge e's q0' / q1' (rows 4e+4, 4e+5) and p1' / p0'
            // (rows 4e+2, 4e+3).  Edge e's q2' is edge e+1's p1 input, which that edge's p1' already
            // carries after the passes; an internal edge's p2' is its neighbour's q1'; only a strong
            // edge 0 writes p2' (row 1: the upper neighbour's row 13).
            tile[4 * e + 4][r] = (uint8_t)o.q0;
            tile[4 * e + 5][r] = (uint8_t)o.q1;
            if (strong0 && e == 0) tile[1][r] = (uint8_t)o.p2;
            tile[4 * e + 2][r] = (uint8_t)o.p1;
            tile[4 * e + 3][r] = (uint8_t)o.p0;
            lds_sync_wave();
            cur = *reinterpret_cast<const uint32_t*>(&tile[4 + r][4 * e]);
            // the upper neighbour's rows 13..15: this row is their writer when it filters its top edge
            if (t0 && r >= 1 && r < 4)
                gst4(Y + (size_t)(mby * 16 - 4 + r) * pitch + 16 * x + 4 * e,
                     *reinterpret_cast<const uint32_t*>(&tile[r][4 * e]));
        }
        // step done: the row above may reuse the ring slot of MB x
        if (!band_first && lane == 0) lds_publish(cons_me, x + 1);
        prev = cur;
        prev_mod = vmod || hmod;
        qprev = qp;
        below_prev = below_cur;
    }
    if (lane == 0) {
        g_db_waits[0][mby][0] = w_cons;
        g_db_waits[0][mby][1] = w_prog;
        g_db_waits[0][mby][2] = w_glb;
    }
    if (lane == 0) lds_store(cons_me, mb_w + 1);
    db_luma_sse(g, fs, rec, G.src_y, mby, lane);
}

// ---------------------------------------------------------------- chroma row engine
// Chroma edges (at chroma columns / rows 0 and 4) modify p0 / q0 only and read p1 / q1, so the two
// edges of a direction never touch each other's samples: one pass, all in parallel.  Vertical
// layout: lane 8k + 2q + c holds line k (0..7) of the MB's 16 interleaved Cb/Cr bytes as dword q
// (chroma columns 2q, 2q+1) and filters component c of the edge whose q side starts in that dword
// (q 0: the MB edge, p side in the left MB's dword 3; q 2: the internal edge, p side in dword 1).
// Horizontal layout: lane 16ce + b filters byte column b (chroma column b / 2, component b % 2) of
// edge ce, reading rows 4ce-2 .. 4ce+1 from a per-wave tile (rows 0..1: the MB above's rows 6..7).
template <int R>
__device__ void db_chroma_row(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                              const int* __restrict__ row_lastq, DbShared<R>& S, const DbGlobal& G, int band_row,
                              int mby, int lane) {
    unsigned long long w_cons = 0, w_prog = 0, w_glb = 0;  // diagnostics: ticks spent waiting
    uint8_t* UV = fs->rec_uv;
    const int pitch = g.pitch, mb_w = g.mb_w;
    const uint32_t epoch = (uint32_t)fs->db_epoch;  // full 32-bit tag above the 32 payload bits
    const bool band_first = band_row == 0, band_last = band_row == R - 1 || mby == g.mb_h - 1;
    const bool pic_last = mby == g.mb_h - 1;
    const int k = lane >> 3, dq4 = (lane >> 1) & 3, comp = lane & 1;  // vertical layout
    const int hb = lane & 15, hce = (lane >> 4) & 1;                   // horizontal layout (lanes < 32)
    int* prog_me = &S.prog[1][band_row];
    int* cons_me = &S.cons[1][band_row];
    uint8_t(*tile)[16] = S.tile[R + band_row];
    const int cqo = fs->chroma_qp_offset;
    const DbLaneTabs T = load_lane_tabs(lane);
    int qrun = __builtin_amdgcn_readfirstlane(row_entry_qp(fs, row_lastq, mby, lane));
    int qprev = qrun;
    uint32_t prev = 0;
    bool prev_mod = false;
    uint32_t pf[kDbPf];
    uint32_t(*stage)[64] = reinterpret_cast<uint32_t(*)[64]>(S.stage[R + band_row]);
    const uint8_t* line = UV + (size_t)(mby * 8 + k) * pitch + 4 * dq4;
    auto issue = [&](int xb) {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j) pf[j] = gld4(line + 16 * min(xb + j, mb_w - 1));
    };
    auto park = [&]() {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j) stage[j][lane] = pf[j];
    };
    issue(0);
    park();
    issue(kDbPf);
    uint32_t cur_nx = stage[0][lane];
    const int cs = 8 * comp;  // bit offset of this component's byte in a dword (bytes c and 2 + c)
    uint4 rb = make_uint4(0, 0, 0, 0);
    uint32_t rbt = 0;
    bool below_prev = false;
    for (int x = 0; x <= mb_w; ++x) {
        const bool have = x < mb_w;
        if (have && (x & 63) == 0) {
            const int xm = min(x + lane, mb_w - 1);
            rb = S.recs[band_row][xm];
            rbt = pic_last ? 0u : (S.recs[band_row + 1][xm].z & 0xfffu);
        }
        uint4 rr = make_uint4(0, 0, 0, 0);
        bool below_cur = false;
        if (have) {
            rr = rd_lane(rb, x & 63);
            below_cur = __builtin_amdgcn_readlane((int)rbt, x & 63) != 0;
        }
        uint32_t cur = cur_nx;
        if ((x + 1) % kDbPf == 0) {
            park();
            issue(x + 1 + kDbPf);
        }
        cur_nx = stage[(x + 1) % kDbPf][lane];
        if (have && (rr.w >> 30) & 1) qrun = (rr.w >> 24) & 63;
        const int qp = qrun;
        const int cq = scqp(T, qp, cqo), cqp = scqp(T, qprev, cqo);
        const DbParams dq = spar(T, cq), dl = spar(T, (cqp + cq + 1) >> 1);
        // ---- vertical chroma edges (luma edges 0 and 2)
        const uint32_t ve0 = rec_edge(rr, 0, 0), ve2 = rec_edge(rr, 0, 2);
        const bool vmod = have && (ve0 | ve2) != 0, v0 = have && ve0 != 0;
        if (vmod) {
            const uint32_t pa = dppmov<kRowShl6>(prev), pb = dppmov<kRowShr2>(cur);
            const uint32_t pw = blend(pa, pb, dq4 == 0);  // p side: the left MB's dword 3 / this MB's dword 1
            const uint32_t b4 = dq4 == 0 ? ve0 : ve2;
            const bool edge_lane = dq4 == 0 || dq4 == 2;
            const int bs = edge_lane ? (int)((b4 >> (3 * (k >> 1))) & 7u) : 0;
            int p1 = (int)((pw >> cs) & 0xff), p0 = (int)((pw >> (16 + cs)) & 0xff);
            int q0 = (int)((cur >> cs) & 0xff);
            const int q1 = (int)((cur >> (16 + cs)) & 0xff);
            db_chroma_line(p1, p0, q0, q1, bs, sel_params(dq4 == 0, dl, dq));
            // this component's bytes of the two dwords; the other component's lane has the rest
            const uint32_t nq = (cur & ~(0xffu << cs)) | ((uint32_t)q0 << cs);
            const uint32_t np = (pw & ~(0xffu << (16 + cs))) | ((uint32_t)p0 << (16 + cs));
            const uint32_t oq = dppmov<kQuadSwap1>(nq), op = dppmov<kQuadSwap1>(np);
            const uint32_t cmask = comp ? 0x00ff00ffu : 0xff00ff00u;  // the other component's bytes
            const uint32_t fq = (nq & ~cmask) | (oq & cmask), fp = (np & ~cmask) | (op & cmask);
            // dword 1 <- edge 2's p side (lane + 2); the left MB's dword 3 <- edge 0's p side (lane - 6)
            const uint32_t from_e2 = dppmov<kRowShl2>(fp), from_e0 = dppmov<kRowShr6>(fp);
            const uint32_t own = blend(fq, cur, edge_lane);
            cur = blend(from_e2, own, dq4 == 1 && ve2 != 0);  // blends, never selects (see the luma engine)
            prev = blend(from_e0, prev, dq4 == 3 && v0);
        }
        if (x > 0) {
            const int xp = x - 1;
            const bool below_top = below_prev;
            if ((prev_mod || v0) && comp == 0 && (k <= 6 || !below_top))
                gst4(UV + (size_t)(mby * 8 + k) * pitch + 16 * xp + 4 * dq4, prev);
            if (below_top) {
                if (!band_last) {
                    const int slot = xp % kDbRing;
                    { const unsigned long long t = wall_clock64(); wait_lds(&S.cons[1][band_row + 1], xp - kDbRing + 1, G.err); w_cons += wall_clock64() - t; }
                    if (k >= 6 && comp == 0)
                        *reinterpret_cast<uint32_t*>(&S.cring[band_row][slot][k - 6][4 * dq4]) = prev;
                    if (lane == 0) S.ringq[1][band_row][slot] = (uint8_t)qprev;
                } else {
                    uint64_t* dst = G.glb + ((size_t)(1 * g.mb_h + mby) * mb_w + xp) * kDbGlbWords;
                    if (k >= 6 && comp == 0) put_tagged(dst + 4 * (k - 6) + dq4, prev, epoch);
                    if (lane == 0) put_tagged(dst + 8, (uint32_t)qprev, epoch);
                }
            }
            if (!band_last && lane == 0) lds_publish(prog_me, x);
        }
        if (!have) break;
        // ---- horizontal chroma edges (luma edges 0 and 2)
        const uint32_t t0 = rec_edge(rr, 1, 0), he2 = rec_edge(rr, 1, 2);
        const bool hmod = (t0 | he2) != 0;
        if (hmod) {
            int qtop = qp;
            if (t0) {  // the row above's bottom chroma rows 6..7 of MB x -> tile rows 0..1
                if (!band_first) {
                    { const unsigned long long t = wall_clock64(); wait_lds(&S.prog[1][band_row - 1], x + 1, G.err); w_prog += wall_clock64() - t; }
                    const int slot = x % kDbRing;
                    if (lane < 8)
                        *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) =
                            *reinterpret_cast<const uint32_t*>(&S.cring[band_row - 1][slot][lane >> 2][4 * (lane & 3)]);
                    qtop = __builtin_amdgcn_readfirstlane(S.ringq[1][band_row - 1][slot]);
                } else {
                    const uint64_t* src = G.glb + ((size_t)(1 * g.mb_h + mby - 1) * mb_w + x) * kDbGlbWords;
                    const unsigned long long tq = wall_clock64();
                    const uint32_t v = poll_tagged(src + (lane <= 8 ? lane : 0), lane <= 8, epoch, G.err);
                    w_glb += wall_clock64() - tq;
                    if (lane < 8) *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) = v;
                    qtop = __builtin_amdgcn_readlane((int)v, 8);
                }
            }
            if (comp == 0) *reinterpret_cast<uint32_t*>(&tile[2 + k][4 * dq4]) = cur;
            const DbParams dt = spar(T, (scqp(T, qtop, cqo) + cq + 1) >> 1);
            lds_sync_wave();
            const bool hl = lane < 32;
            const int r0 = 4 * hce;  // tile rows r0 .. r0+3 = p1, p0, q0, q1
            int p1 = tile[r0][hb], p0 = tile[r0 + 1][hb], q0 = tile[r0 + 2][hb];
            const int q1 = tile[r0 + 3][hb];
            const uint32_t b4 = hce ? he2 : t0;
            const int bs = hl ? (int)((b4 >> (3 * (hb >> 2))) & 7u) : 0;
            db_chroma_line(p1, p0, q0, q1, bs, sel_params(hce == 0, dt, dq));
            lds_sync_wave();
            if (hl) {
                tile[r0 + 1][hb] = (uint8_t)p0;
                tile[r0 + 2][hb] = (uint8_t)q0;
            }
            lds_sync_wave();
            cur = *reinterpret_cast<const uint32_t*>(&tile[2 + k][4 * dq4]);
            if (t0 && lane < 4)  // the upper neighbour's row 7
                gst4(UV + (size_t)(mby * 8 - 1) * pitch + 16 * x + 4 * lane,
                     *reinterpret_cast<const uint32_t*>(&tile[1][4 * lane]));
            lds_sync_wave();
        }
        if (!band_first && lane == 0) lds_publish(cons_me, x + 1);
        prev = cur;
        prev_mod = vmod || hmod;
        qprev = qp;
        below_prev = below_cur;
    }
    if (lane == 0) {
        g_db_waits[1][mby][0] = w_cons;
        g_db_waits[1][mby][1] = w_prog;
        g_db_waits[1][mby][2] = w_glb;
    }
    if (lane == 0) lds_store(cons_me, mb_w + 1);
    db_chroma_sse(g, fs, rec, G.src_uv, mby, lane);
}

template <int R>
__global__ __launch_bounds__(64 * R) void k_deblock(Geometry g, const FrameState* __restrict__ fs,
                                                          const uint4* __restrict__ rec,
                                                          const int* __restrict__ row_lastq, DbGlobal G) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    // one workgroup per (band, plane): 8 waves of 512 threads leave each wave 256 VGPRs for the
    // line registers and the prefetch batch
    __shared__ DbShared<R> S;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int band_row = wave, plane = blockIdx.y;
    if (threadIdx.x < 2 * R) {
        S.prog[threadIdx.x / R][threadIdx.x % R] = 0;
        S.cons[threadIdx.x / R][threadIdx.x % R] = 0;
    }
    if (threadIdx.x < 52) {
        const DbParams d = db_params((int)threadIdx.x);
        S.params[threadIdx.x] = (uint32_t)d.alpha | ((uint32_t)d.beta << 8) | (d.tc0 << 13);
        S.cqp[threadIdx.x] = (uint8_t)chroma_qp((int)threadIdx.x, 0);
    }
    {  // the band's records and the next row's (their top-edge bS decides who writes rows 13..15)
        const int r0 = blockIdx.x * R, nrow = min(R + 1, g.mb_h - r0);
        for (int i = threadIdx.x; i < nrow * g.mb_w; i += blockDim.x) {
            const int rr = i / g.mb_w, xx = i - rr * g.mb_w;
            S.recs[rr][xx] = rec[(size_t)(r0 + rr) * g.mb_w + xx];
        }
    }
    __syncthreads();
    const int mby = blockIdx.x * R + band_row;
    if (mby >= g.mb_h) return;  // no row above a missing row waits on it (rows below are missing too)
    const unsigned long long t_start = wall_clock64(), c_start = __builtin_amdgcn_s_memtime();
    if (plane == 0)
        db_luma_row<R>(g, fs, rec, row_lastq, S, G, band_row, mby, lane);
    else
        db_chroma_row<R>(g, fs, rec, row_lastq, S, G, band_row, mby, lane);
    if (lane == 0) {
        g_db_stamps[plane][mby][0] = t_start;
        g_db_stamps[plane][mby][1] = wall_clock64();
        g_db_clk[plane][mby] = __builtin_amdgcn_s_memtime() - c_start;
    }
}

}  // namespace

std::vector<unsigned long long> deblock_row_stamps(int mb_h) {
    std::vector<unsigned long long> v((size_t)2 * kMaxSlices * 2), w((size_t)2 * kMaxSlices * 3);
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_db_stamps), v.size() * sizeof(unsigned long long)));
    HIP_CHECK(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_db_waits), w.size() * sizeof(unsigned long long)));
    std::vector<unsigned long long> ph((size_t)kMaxSlices * 4);
    HIP_CHECK(hipMemcpyFromSymbol(ph.data(), HIP_SYMBOL(g_db_phase), ph.size() * sizeof(unsigned long long)));
    std::vector<unsigned long long> out;  // per plane and row: start, end, wait ring, wait above, wait band
    for (int p = 0; p < 2; ++p)
        for (int y = 0; y < mb_h; ++y) {
            out.push_back(v[((size_t)p * kMaxSlices + y) * 2]);
            out.push_back(v[((size_t)p * kMaxSlices + y) * 2 + 1]);
            for (int k = 0; k < 3; ++k) out.push_back(w[((size_t)p * kMaxSlices + y) * 3 + k]);
        }
    for (int y = 0; y < mb_h; ++y)  // then the luma rows' phase ticks: head, V, final, H
        for (int k = 0; k < 4; ++k) out.push_back(ph[(size_t)y * 4 + k]);
    std::vector<unsigned long long> ck((size_t)2 * kMaxSlices);
    HIP_CHECK(hipMemcpyFromSymbol(ck.data(), HIP_SYMBOL(g_db_clk), ck.size() * sizeof(unsigned long long)));
    for (int p = 0; p < 2; ++p)  // then each row wave's shader-clock cycles
        for (int y = 0; y < mb_h; ++y) out.push_back(ck[(size_t)p * kMaxSlices + y]);
    return out;
}

void launch_deblock(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                    hipStream_t stream) {
    if (g.mb_w > kDbMaxW || g.mb_h > kMaxSlices) throw std::invalid_argument("launch_deblock: picture too large");
    hipLaunchKernelGGL(k_db_prep, dim3(g.mb_h), dim3(256), 0, stream, g, b.fs, b.mb, b.db_rec, b.db_rowq);
    DbGlobal G{b.db_glb, b.db_err, src_y, src_uv};
    static const int rows = [] {
        const char* e = std::getenv("MXDESK_DB_ROWS");
        return e && std::atoi(e) == 8 ? 8 : (e && std::atoi(e) == 4 ? 4 : kDbRowsDefault);
    }();
    if (rows == 8)
        hipLaunchKernelGGL(k_deblock<8>, dim3((g.mb_h + 7) / 8, 2), dim3(64 * 8), 0, stream, g, b.fs, b.db_rec, b.db_rowq, G);
    else
        hipLaunchKernelGGL(k_deblock<4>, dim3((g.mb_h + 3) / 4, 2), dim3(64 * 4), 0, stream, g, b.fs, b.db_rec, b.db_rowq, G);
    // (the filtered picture's distortion is summed by k_deblock's row waves: no k_db_sse pass)
}

}  // namespace h264
}  // namespace mx
