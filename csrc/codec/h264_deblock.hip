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
//    left to right; 8 rows x 2 planes = 16 waves per workgroup.  A lane owns one sample line: the
//    vertical edges run on lines in registers, the horizontal edges on columns after a transpose
//    through a per-wave LDS tile.  A row hands each finished macroblock's bottom lines (luma rows
//    12..15, chroma rows 6..7: the p samples of the next row's top edge) down through an LDS ring
//    with a progress counter (the row below waits only where its own top edge is filtered); the
//    band's last row hands them to the next workgroup (another XCD, another L2) through global
//    memory as epoch-tagged 64-bit agent-scope atomic words -- 32 sample bits and the frame's tag
//    -- which the consumer polls directly: no agent-scope release fence per macroblock (on gfx950
//    a write-back of the XCD's whole L2, which set the pace of every row below the band).
//    Every sample byte has exactly one writer: rows 13..15 of a macroblock whose lower neighbour
//    filters its top edge are written by the row below, else by their own row.
//    Macroblocks with every bS == 0 (static desktop, skips with equal vectors) cost a record read
//    and a counter update, so P pictures pay for the changing areas only.
//  * k_db_sse: the distortion of the filtered picture (one partial per MB row and channel), which
//    replaces the analysis kernels' unfiltered figures in the frame statistics.
#include <hip/hip_runtime.h>

#include "../common/hip_check.h"
#include "h264_deblock.h"
#include "h264_gpu.h"
#include "h264_mb.h"

namespace mx {
namespace h264 {

namespace {

constexpr int kDbRows = 8;   // MB rows (waves per plane) per workgroup
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

struct DbShared {
    uint8_t lring[kDbRows][kDbRing][4][16];  // luma rows 12..15 of a finished MB
    uint8_t cring[kDbRows][kDbRing][2][16];  // chroma rows 6..7 (interleaved U/V)
    uint8_t ringq[2][kDbRows][kDbRing];      // the MB's QP_Y (per plane's own running value)
    int prog[2][kDbRows];                    // ring entries published (MB count)
    int cons[2][kDbRows];                    // MB steps finished by the row (for the row above's ring reuse)
    uint8_t tile[2 * kDbRows][20][16];       // per-wave transposition tile
    uint4 recs[kDbRows + 1][kDbMaxW];        // the band's records + the next row's (bS, QP)
    uint4 stage[2 * kDbRows][kDbPf][16];     // per-wave prefetched sample lines (lane-private slots)
    uint32_t params[52];                     // alpha | beta << 8 | packed tC0 << 13, by indexA
    uint8_t cqp[52];                         // QP_C of a clipped qP_I (Table 8-15)
};
__device__ __forceinline__ int lds_cqp(const DbShared& S, int qp, int offset) {
    const int q = qp + offset;
    return S.cqp[q < 0 ? 0 : (q > 51 ? 51 : q)];
}
__device__ __forceinline__ DbParams lds_params(const DbShared& S, int qpav) {
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

// ---------------------------------------------------------------- luma row engine
__device__ void db_luma_row(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                            const int* __restrict__ row_lastq, DbShared& S, const DbGlobal& G, int band_row,
                            int mby, int lane) {
    uint8_t* Y = fs->rec_y;
    const int pitch = g.pitch, mb_w = g.mb_w;
    const uint32_t epoch = (uint32_t)fs->db_epoch;  // full 32-bit tag above the 32 payload bits
    const bool band_first = band_row == 0, band_last = band_row == kDbRows - 1 || mby == g.mb_h - 1;
    const bool pic_last = mby == g.mb_h - 1;
    const bool act = lane < 16;
    int* prog_me = &S.prog[0][band_row];
    int* cons_me = &S.cons[0][band_row];
    uint8_t(*tile)[16] = S.tile[band_row];
    int qrun = row_entry_qp(fs, row_lastq, mby, lane);
    int qprev = qrun;           // QP_Y of MB x-1
    int P[16], C[16];           // MB x-1 (row `lane`, post-H) and MB x (row `lane`)
    bool prev_mod = false;      // MB x-1 was modified (its own edges)
    for (int k = 0; k < 16; ++k) P[k] = 0;
    // sample lines: batches of kDbPf macroblocks loaded one batch ahead into registers and parked in
    // the wave's LDS stage when their batch starts, so a load's latency spans kDbPf steps
    uint4 pf[kDbPf];
    uint4(*stage)[16] = S.stage[band_row];
    const uint8_t* line = Y + (size_t)(mby * 16 + (act ? lane : 0)) * pitch;
    auto issue = [&](int xb) {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j)
            pf[j] = gld16(line + 16 * min(xb + j, mb_w - 1));  // unconditional: a select on the
                                                               // loaded value would wait for it here
    };
    issue(0);
    for (int x = 0; x <= mb_w; ++x) {
        const bool have = x < mb_w;
        if (x % kDbPf == 0) {
            if (act) {
#pragma unroll
                for (int j = 0; j < kDbPf; ++j) stage[j][lane] = pf[j];
            }
            issue(x + kDbPf);
        }
        uint4 r = make_uint4(0, 0, 0, 0);
        if (have) {
            if (act) unpack16(stage[x % kDbPf][lane], C);
            r = S.recs[band_row][x];
        }
        if (have && (r.w >> 30) & 1) qrun = (r.w >> 24) & 63;
        const int qp = qrun;
        // ---- vertical edges of MB x (lines); edge 0 also finishes MB x-1's columns 13..15
        bool vmod = false, v0 = false;
        // the MB's filter parameters: its own QP (internal edges, and the horizontal ones) and the
        // left edge's average -- both fetched before the edges, one LDS round trip
        const DbParams dq = lds_params(S, qp), dl = lds_params(S, (qprev + qp + 1) >> 1);
        if (have) {
            for (int e = 0; e < 4; ++e) {
                const uint32_t b4 = rec_edge(r, 0, e);
                if (!b4) continue;
                vmod = true;
                const int bs = (b4 >> (3 * (lane >> 2))) & 7;
                const DbParams d = e == 0 ? dl : dq;
                if (e == 0) {
                    v0 = true;
                    if (act) db_luma_line(P[12], P[13], P[14], P[15], C[0], C[1], C[2], C[3], bs, d);
                } else if (e == 1) {
                    if (act) db_luma_line(C[0], C[1], C[2], C[3], C[4], C[5], C[6], C[7], bs, d);
                } else if (e == 2) {
                    if (act) db_luma_line(C[4], C[5], C[6], C[7], C[8], C[9], C[10], C[11], bs, d);
                } else {
                    if (act) db_luma_line(C[8], C[9], C[10], C[11], C[12], C[13], C[14], C[15], bs, d);
                }
            }
        }
        // ---- MB x-1 is final (except rows 13..15 when the row below filters its top edge there)
        if (x > 0) {
            const int xp = x - 1;
            const bool below_top = !pic_last && rec_edge(S.recs[band_row + 1][xp], 1, 0) != 0;
            if ((prev_mod || v0) && act && (lane <= 12 || !below_top))
                gst16(Y + (size_t)(mby * 16 + lane) * pitch + 16 * xp, pack16(P));
            if (below_top) {
                if (!band_last) {
                    const int slot = xp % kDbRing;
                    wait_lds(&S.cons[0][band_row + 1], xp - kDbRing + 1, G.err);  // ring slot free
                    if (lane >= 12 && act)
                        *reinterpret_cast<uint4*>(S.lring[band_row][slot][lane - 12]) = pack16(P);
                    if (lane == 0) S.ringq[0][band_row][slot] = (uint8_t)qprev;
                } else {
                    uint64_t* dst = G.glb + ((size_t)(0 * g.mb_h + mby) * mb_w + xp) * kDbGlbWords;
                    if (lane >= 12 && act) {
                        const uint4 v = pack16(P);
                        put_tagged(dst + 4 * (lane - 12), v.x, epoch);
                        put_tagged(dst + 4 * (lane - 12) + 1, v.y, epoch);
                        put_tagged(dst + 4 * (lane - 12) + 2, v.z, epoch);
                        put_tagged(dst + 4 * (lane - 12) + 3, v.w, epoch);
                    }
                    if (lane == 0) put_tagged(dst + kDbQWord, (uint32_t)qprev, epoch);
                }
            }
            if (!band_last) {
                lds_sync_wave();
                if (lane == 0) lds_store(prog_me, x);
            }
        }
        if (!have) break;
        // ---- horizontal edges of MB x (columns, after a transpose through the tile)
        const uint32_t t0 = rec_edge(r, 1, 0);
        bool hmod = false;
        for (int e = 0; e < 4; ++e) hmod |= rec_edge(r, 1, e) != 0;
        if (hmod) {
            int qtop = qp;
            if (t0) {  // the row above's bottom lines of MB x
                if (!band_first) {
                    wait_lds(&S.prog[0][band_row - 1], x + 1, G.err);
                    const int slot = x % kDbRing;
                    if (lane < 4)
                        *reinterpret_cast<uint4*>(tile[lane]) =
                            *reinterpret_cast<const uint4*>(S.lring[band_row - 1][slot][lane]);
                    qtop = S.ringq[0][band_row - 1][slot];
                } else {
                    // rows 12..15 of the band above (lanes 0..15, a word each) and its QP_Y (lane 16);
                    // the poll retires its loads here (left pending, the compiler's wait at the merge
                    // below would be a vmcnt(0) on every row's H phase)
                    const uint64_t* src = G.glb + ((size_t)(0 * g.mb_h + mby - 1) * mb_w + x) * kDbGlbWords;
                    const uint32_t v = poll_tagged(src + (lane <= kDbQWord ? lane : 0), lane <= kDbQWord, epoch, G.err);
                    if (lane < 16) *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) = v;
                    qtop = __builtin_amdgcn_readlane((int)v, kDbQWord);
                }
            }
            if (act) *reinterpret_cast<uint4*>(tile[4 + lane]) = pack16(C);
            const DbParams dt = lds_params(S, (qtop + qp + 1) >> 1);
            lds_sync_wave();
            int col[20];
            if (act) {
#pragma unroll
                for (int k = 0; k < 20; ++k) col[k] = tile[k][lane];
            }
            for (int e = 0; e < 4; ++e) {
                const uint32_t b4 = rec_edge(r, 1, e);
                if (!b4) continue;
                const int bs = (b4 >> (3 * (lane >> 2))) & 7;
                const DbParams d = e == 0 ? dt : dq;
                if (!act) continue;
                if (e == 0)
                    db_luma_line(col[0], col[1], col[2], col[3], col[4], col[5], col[6], col[7], bs, d);
                else if (e == 1)
                    db_luma_line(col[4], col[5], col[6], col[7], col[8], col[9], col[10], col[11], bs, d);
                else if (e == 2)
                    db_luma_line(col[8], col[9], col[10], col[11], col[12], col[13], col[14], col[15], bs, d);
                else
                    db_luma_line(col[12], col[13], col[14], col[15], col[16], col[17], col[18], col[19], bs, d);
            }
            if (act) {
#pragma unroll
                for (int k = 1; k < 20; ++k) tile[k][lane] = (uint8_t)col[k];
            }
            lds_sync_wave();
            if (act) unpack16(*reinterpret_cast<const uint4*>(tile[4 + lane]), C);
            // the upper neighbour's rows 13..15: this row is their writer when it filters its top edge
            if (t0 && lane >= 1 && lane < 4)
                gst16(Y + (size_t)(mby * 16 - 4 + lane) * pitch + 16 * x, *reinterpret_cast<const uint4*>(tile[lane]));
        }
        // step done: the row above may reuse the ring slot of MB x
        if (!band_first && lane == 0) lds_store(cons_me, x + 1);
#pragma unroll
        for (int k = 0; k < 16; ++k) P[k] = C[k];
        prev_mod = vmod || hmod;
        qprev = qp;
    }
    if (lane == 0) lds_store(cons_me, mb_w + 1);
}

// ---------------------------------------------------------------- chroma row engine
// lane l < 16: component l >> 3 (0 = Cb, 1 = Cr), line / column l & 7
__device__ void db_chroma_row(const Geometry& g, const FrameState* fs, const uint4* __restrict__ rec,
                              const int* __restrict__ row_lastq, DbShared& S, const DbGlobal& G, int band_row,
                              int mby, int lane) {
    uint8_t* UV = fs->rec_uv;
    const int pitch = g.pitch, mb_w = g.mb_w;
    const uint32_t epoch = (uint32_t)fs->db_epoch;  // full 32-bit tag above the 32 payload bits
    const bool band_first = band_row == 0, band_last = band_row == kDbRows - 1 || mby == g.mb_h - 1;
    const bool pic_last = mby == g.mb_h - 1;
    const bool act = lane < 16;
    const int comp = (lane >> 3) & 1, ln = lane & 7;
    int* prog_me = &S.prog[1][band_row];
    int* cons_me = &S.cons[1][band_row];
    uint8_t(*tile)[16] = S.tile[kDbRows + band_row];
    const int cqo = fs->chroma_qp_offset;
    int qrun = row_entry_qp(fs, row_lastq, mby, lane);
    int qprev = qrun;
    int P[8], C[8];
    bool prev_mod = false;
    for (int k = 0; k < 8; ++k) P[k] = 0;
    auto load_line = [&](const uint4& v, int* o) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (w[k >> 1] >> (16 * (k & 1) + 8 * comp)) & 0xff;
    };
    // write this lane's 8 samples into tile row `row` (interleaved with the other component)
    auto to_tile = [&](int row, const int* o) {
#pragma unroll
        for (int k = 0; k < 8; ++k) tile[row][2 * k + comp] = (uint8_t)o[k];
    };
    uint4 pf[kDbPf];
    uint4(*stage)[16] = S.stage[kDbRows + band_row];
    const uint8_t* line = UV + (size_t)(mby * 8 + ln) * pitch;
    auto issue = [&](int xb) {
#pragma unroll
        for (int j = 0; j < kDbPf; ++j)
            pf[j] = gld16(line + 16 * min(xb + j, mb_w - 1));  // unconditional: a select on the
                                                               // loaded value would wait for it here
    };
    issue(0);
    for (int x = 0; x <= mb_w; ++x) {
        const bool have = x < mb_w;
        if (x % kDbPf == 0) {
            if (act) {
#pragma unroll
                for (int j = 0; j < kDbPf; ++j) stage[j][lane] = pf[j];
            }
            issue(x + kDbPf);
        }
        uint4 r = make_uint4(0, 0, 0, 0);
        if (have) {
            if (act) load_line(stage[x % kDbPf][lane], C);
            r = S.recs[band_row][x];
        }
        if (have && (r.w >> 30) & 1) qrun = (r.w >> 24) & 63;
        const int qp = qrun;
        bool vmod = false, v0 = false;
        const int cq = lds_cqp(S, qp, cqo), cqp = lds_cqp(S, qprev, cqo);
        const DbParams dq = lds_params(S, cq), dl = lds_params(S, (cqp + cq + 1) >> 1);
        if (have) {
            for (int ce = 0; ce < 2; ++ce) {
                const uint32_t b4 = rec_edge(r, 0, 2 * ce);
                if (!b4) continue;
                vmod = true;
                const int bs = (b4 >> (3 * (ln >> 1))) & 7;
                const DbParams d = ce == 0 ? dl : dq;
                if (ce == 0) {
                    v0 = true;
                    if (act) db_chroma_line(P[6], P[7], C[0], C[1], bs, d);
                } else if (act) {
                    db_chroma_line(C[2], C[3], C[4], C[5], bs, d);
                }
            }
        }
        if (x > 0) {
            const int xp = x - 1;
            const bool below_top = !pic_last && rec_edge(S.recs[band_row + 1][xp], 1, 0) != 0;
            if (prev_mod || v0 || below_top) {
                // MB x-1's rows through the tile (the two components interleave)
                if (act) to_tile(2 + ln, P);
                lds_sync_wave();
                if ((prev_mod || v0) && lane < 8 && (lane <= 6 || !below_top))
                    gst16(UV + (size_t)(mby * 8 + lane) * pitch + 16 * xp, *reinterpret_cast<const uint4*>(tile[2 + lane]));
                if (below_top) {
                    if (!band_last) {
                        const int slot = xp % kDbRing;
                        wait_lds(&S.cons[1][band_row + 1], xp - kDbRing + 1, G.err);
                        if (lane < 2)
                            *reinterpret_cast<uint4*>(S.cring[band_row][slot][lane]) =
                                *reinterpret_cast<const uint4*>(tile[8 + lane]);
                        if (lane == 0) S.ringq[1][band_row][slot] = (uint8_t)qprev;
                    } else {
                        uint64_t* dst = G.glb + ((size_t)(1 * g.mb_h + mby) * mb_w + xp) * kDbGlbWords;
                        if (lane < 8)
                            put_tagged(dst + lane, *reinterpret_cast<const uint32_t*>(&tile[8 + (lane >> 2)][4 * (lane & 3)]),
                                       epoch);
                        if (lane == 0) put_tagged(dst + 8, (uint32_t)qprev, epoch);
                    }
                }
                lds_sync_wave();  // tile reads done before it is rewritten
            }
            if (!band_last) {
                lds_sync_wave();
                if (lane == 0) lds_store(prog_me, x);
            }
        }
        if (!have) break;
        const uint32_t t0 = rec_edge(r, 1, 0);
        const bool hmod = t0 != 0 || rec_edge(r, 1, 2) != 0;
        if (hmod) {
            int qtop = qp;
            if (t0) {
                if (!band_first) {
                    wait_lds(&S.prog[1][band_row - 1], x + 1, G.err);
                    const int slot = x % kDbRing;
                    if (lane < 2)
                        *reinterpret_cast<uint4*>(tile[lane]) =
                            *reinterpret_cast<const uint4*>(S.cring[band_row - 1][slot][lane]);
                    qtop = S.ringq[1][band_row - 1][slot];
                } else {
                    const uint64_t* src = G.glb + ((size_t)(1 * g.mb_h + mby - 1) * mb_w + x) * kDbGlbWords;
                    const uint32_t v = poll_tagged(src + (lane <= 8 ? lane : 0), lane <= 8, epoch, G.err);
                    if (lane < 8) *reinterpret_cast<uint32_t*>(&tile[lane >> 2][4 * (lane & 3)]) = v;
                    qtop = __builtin_amdgcn_readlane((int)v, 8);
                }
            }
            if (act) to_tile(2 + ln, C);
            const DbParams dt = lds_params(S, (lds_cqp(S, qtop, cqo) + cq + 1) >> 1);
            lds_sync_wave();
            int col[10];
            if (act) {
#pragma unroll
                for (int k = 0; k < 10; ++k) col[k] = tile[k][2 * ln + comp];
            }
            for (int ce = 0; ce < 2; ++ce) {
                const uint32_t b4 = rec_edge(r, 1, 2 * ce);
                if (!b4) continue;
                const int bs = (b4 >> (3 * (ln >> 1))) & 7;
                const DbParams d = ce == 0 ? dt : dq;
                if (!act) continue;
                if (ce == 0)
                    db_chroma_line(col[0], col[1], col[2], col[3], bs, d);
                else
                    db_chroma_line(col[4], col[5], col[6], col[7], bs, d);
            }
            if (act) {
#pragma unroll
                for (int k = 1; k < 10; ++k) tile[k][2 * ln + comp] = (uint8_t)col[k];
            }
            lds_sync_wave();
            if (act) {
#pragma unroll
                for (int k = 0; k < 8; ++k) C[k] = tile[2 + ln][2 * k + comp];
            }
            if (t0 && lane == 1)  // the upper neighbour's row 7
                gst16(UV + (size_t)(mby * 8 - 1) * pitch + 16 * x, *reinterpret_cast<const uint4*>(tile[1]));
            lds_sync_wave();
        }
        if (!band_first && lane == 0) lds_store(cons_me, x + 1);
#pragma unroll
        for (int k = 0; k < 8; ++k) P[k] = C[k];
        prev_mod = vmod || hmod;
        qprev = qp;
    }
    if (lane == 0) lds_store(cons_me, mb_w + 1);
}

__global__ __launch_bounds__(64 * kDbRows) void k_deblock(Geometry g, const FrameState* __restrict__ fs,
                                                          const uint4* __restrict__ rec,
                                                          const int* __restrict__ row_lastq, DbGlobal G) {
    // a serial chain on few waves: issue priority over the bulk kernels sharing its SIMDs
    __builtin_amdgcn_s_setprio(3);
    // one workgroup per (band, plane): 8 waves of 512 threads leave each wave 256 VGPRs for the
    // line registers and the prefetch batch
    __shared__ DbShared S;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int band_row = wave, plane = blockIdx.y;
    if (threadIdx.x < 2 * kDbRows) {
        S.prog[threadIdx.x / kDbRows][threadIdx.x % kDbRows] = 0;
        S.cons[threadIdx.x / kDbRows][threadIdx.x % kDbRows] = 0;
    }
    if (threadIdx.x < 52) {
        const DbParams d = db_params((int)threadIdx.x);
        S.params[threadIdx.x] = (uint32_t)d.alpha | ((uint32_t)d.beta << 8) | (d.tc0 << 13);
        S.cqp[threadIdx.x] = (uint8_t)chroma_qp((int)threadIdx.x, 0);
    }
    {  // the band's records and the next row's (their top-edge bS decides who writes rows 13..15)
        const int r0 = blockIdx.x * kDbRows, nrow = min(kDbRows + 1, g.mb_h - r0);
        for (int i = threadIdx.x; i < nrow * g.mb_w; i += blockDim.x) {
            const int rr = i / g.mb_w, xx = i - rr * g.mb_w;
            S.recs[rr][xx] = rec[(size_t)(r0 + rr) * g.mb_w + xx];
        }
    }
    __syncthreads();
    const int mby = blockIdx.x * kDbRows + band_row;
    if (mby >= g.mb_h) return;  // no row above a missing row waits on it (rows below are missing too)
    if (plane == 0)
        db_luma_row(g, fs, rec, row_lastq, S, G, band_row, mby, lane);
    else
        db_chroma_row(g, fs, rec, row_lastq, S, G, band_row, mby, lane);
}

// Distortion of the filtered picture: one workgroup per MB row, partials Y, U, V, Y outside the
// quality mask (sse_part[c][row]; k_scan_rows takes mb_h partials when the filter is on).
__global__ __launch_bounds__(256) void k_db_sse(Geometry g, const FrameState* __restrict__ fs,
                                                const uint8_t* __restrict__ src_y, const uint8_t* __restrict__ src_uv) {
    const int mby = blockIdx.x;
    unsigned long long sy = 0, su = 0, sv = 0, sm = 0;
    const int nchunk = g.mb_w * 16;  // 4-byte chunks in 16 rows of a MB row (luma)
    for (int c = threadIdx.x; c < nchunk * 4; c += 256) {
        const int row = c / (g.mb_w * 4), x4 = (c % (g.mb_w * 4)) * 4;
        const int yy = mby * 16 + row;
        if (yy >= g.height || x4 >= g.width) continue;
        const uint32_t a = *reinterpret_cast<const uint32_t*>(src_y + (size_t)yy * g.pitch + x4);
        const uint32_t b = *reinterpret_cast<const uint32_t*>(fs->rec_y + (size_t)yy * g.pitch + x4);
        unsigned s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (int)((a >> (8 * k)) & 0xff) - (int)((b >> (8 * k)) & 0xff);
            s += (x4 + k < g.width) ? (unsigned)(d * d) : 0u;
        }
        sy += s;
        if (mb_unmasked(fs, x4 >> 4, mby)) sm += s;
    }
    for (int c = threadIdx.x; c < g.mb_w * 4 * 8; c += 256) {  // 8 chroma rows, 4-byte chunks (2 U + 2 V)
        const int row = c / (g.mb_w * 4), x4 = (c % (g.mb_w * 4)) * 4;
        const int yy = mby * 8 + row;
        if (2 * yy >= g.height || x4 >= g.width) continue;
        const uint32_t a = *reinterpret_cast<const uint32_t*>(src_uv + (size_t)yy * g.pitch + x4);
        const uint32_t b = *reinterpret_cast<const uint32_t*>(fs->rec_uv + (size_t)yy * g.pitch + x4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (int)((a >> (8 * k)) & 0xff) - (int)((b >> (8 * k)) & 0xff);
            const unsigned e = (x4 + k < g.width) ? (unsigned)(d * d) : 0u;
            if (k & 1) sv += e; else su += e;
        }
    }
    __shared__ unsigned long long part[4][4];
    unsigned long long v[4] = {sy, su, sv, sm};
    for (int c = 0; c < 4; ++c)
        for (int o = 32; o > 0; o >>= 1) v[c] += __shfl_xor(v[c], o, 64);
    if ((threadIdx.x & 63) == 0)
        for (int c = 0; c < 4; ++c) part[c][threadIdx.x >> 6] = v[c];
    __syncthreads();
    if (threadIdx.x < 4) {
        const int c = threadIdx.x;
        fs->sse_part[c * kSsePartStride + mby] = part[c][0] + part[c][1] + part[c][2] + part[c][3];
    }
}

}  // namespace

void launch_deblock(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                    hipStream_t stream) {
    if (g.mb_w > kDbMaxW || g.mb_h > kMaxSlices) throw std::invalid_argument("launch_deblock: picture too large");
    hipLaunchKernelGGL(k_db_prep, dim3(g.mb_h), dim3(256), 0, stream, g, b.fs, b.mb, b.db_rec, b.db_rowq);
    DbGlobal G{b.db_glb, b.db_err};
    hipLaunchKernelGGL(k_deblock, dim3((g.mb_h + kDbRows - 1) / kDbRows, 2), dim3(64 * kDbRows), 0, stream, g, b.fs,
                       b.db_rec, b.db_rowq, G);
    hipLaunchKernelGGL(k_db_sse, dim3(g.mb_h), dim3(256), 0, stream, g, b.fs, src_y, src_uv);
}

}  // namespace h264
}  // namespace mx
