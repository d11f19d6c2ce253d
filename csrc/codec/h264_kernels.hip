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
//  * k_intra_rows   one wave per MB row (slice per row): Intra16x16 H/DC with a serial
//                   left-to-right dependency held in LDS.
//  * k_cavlc        one wave per macroblock: lane 0 codes the MB header (P_Skip decision,
//                   median mv prediction, cbp), lanes 1..27 code one residual block each;
//                   a wave prefix-sum places every lane's bits in an LDS slot.
//  * k_scan         one workgroup: skip runs, per-MB and per-slice bit offsets.
//  * k_pack         one wave per MB / slice: OR the slot bits into the payload.
//  * k_copy_out     payload -> pinned host memory (zero-copy), exactly total_bytes.
#include <hip/hip_runtime.h>

#include "h264_core.h"
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

    __device__ void init(uint32_t* d, uint32_t bitpos) {
        dst = d;
        pos = bitpos;
        acc = 0;
        nacc = 0;
        bits = 0;
    }
    __device__ void emit(uint32_t w, int n) {  // w: n valid bits left-aligned
        const uint32_t wi = pos >> 5, sh = pos & 31;
        uint32_t a = w >> sh;
        if (a) atomicOr(dst + wi, kSwap ? bswap32(a) : a);
        if (sh && n > (int)(32 - sh)) {
            uint32_t b2 = w << (32 - sh);
            if (b2) atomicOr(dst + wi + 1, kSwap ? bswap32(b2) : b2);
        }
        pos += n;
    }
    __device__ void put(uint32_t v, int n) {
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
    __device__ void flush() {
        if (nacc > 0) {
            emit((uint32_t)(acc << (32 - nacc)), nacc);
            nacc = 0;
            acc = 0;
        }
    }
};

__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------------ motion estimation
constexpr int kMaxRange = 32;
constexpr int kWinStride = 16 + 2 * kMaxRange + 8;  // bytes per LDS window row (dword padded)

__global__ __launch_bounds__(256) void k_me_full(Geometry g, const FrameState* __restrict__ fs,
                                                  const uint8_t* __restrict__ src_y, MbInfo* __restrict__ mbs) {
    __shared__ uint32_t win32[(16 + 2 * kMaxRange) * kWinStride / 4];
    __shared__ uint32_t srcw[64];
    __shared__ unsigned long long red[4];
    __shared__ int sub_cost[9];

    const int mbi = blockIdx.x;
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    const int x0 = mbx * 16, y0 = mby * 16;
    const int tid = threadIdx.x;
    int R = fs->search_range;
    R = R > kMaxRange ? kMaxRange : (R < 1 ? 1 : R);
    const int W = 16 + 2 * R;
    const uint8_t* ref = fs->ref_y;
    const int qp = fs->qp;
    const int lambda = lambda_sad(qp);

    uint8_t* win = reinterpret_cast<uint8_t*>(win32);
    for (int i = tid; i < W * kWinStride; i += 256) {
        const int wy = i / kWinStride, wx = i - wy * kWinStride;
        win[i] = (wx < W) ? (uint8_t)ref_px(ref, g.pitch, g.coded_w, g.coded_h, x0 - R + wx, y0 - R + wy) : 0;
    }
    if (tid < 64) {
        const int r = tid >> 2, c = (tid & 3) * 4;
        srcw[tid] = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c);
    }
    __syncthreads();

    const int side = 2 * R + 1, ncand = side * side;
    unsigned long long best = ~0ull;
    for (int c = tid; c < ncand; c += 256) {
        const int dy = c / side - R, dx = c - (c / side) * side - R;
        uint32_t sad = 0;
#pragma unroll 4
        for (int r = 0; r < 16; ++r) {
            const int base = (dy + R + r) * kWinStride + (dx + R);
            const int a = base >> 2, sh = base & 3;
            const uint32_t w0 = win32[a], w1 = win32[a + 1], w2 = win32[a + 2], w3 = win32[a + 3], w4 = win32[a + 4];
            sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, sh), srcw[r * 4 + 0], sad);
            sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w2, w1, sh), srcw[r * 4 + 1], sad);
            sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w3, w2, sh), srcw[r * 4 + 2], sad);
            sad = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w4, w3, sh), srcw[r * 4 + 3], sad);
        }
        const uint32_t cost = me_cost(sad, lambda, 4 * dx, 4 * dy);
        const uint32_t dist = (uint32_t)(abs(dx) + abs(dy));
        const unsigned long long key = ((unsigned long long)cost << 32) | (dist << 16) | (uint32_t)c;
        best = key < best ? key : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long other = __shfl_xor(best, o, 64);
        best = other < best ? other : best;
    }
    if ((tid & 63) == 0) red[tid >> 6] = best;
    __syncthreads();
    unsigned long long b = red[0];
    for (int i = 1; i < 4; ++i) b = red[i] < b ? red[i] : b;
    const int cbest = (int)(b & 0xffff);
    int mvx = 4 * ((cbest % side) - R), mvy = 4 * ((cbest / side) - R);

    if (fs->subpel) {
        // two refinement rounds: half-pel (step 2) then quarter-pel (step 1), 8 neighbours each.
        const int px = tid & 15, py = tid >> 4;
        const int s = src_y[(y0 + py) * g.pitch + x0 + px];
        uint32_t cur_cost;
        {
            const int p = luma_qpel(ref, g.pitch, g.coded_w, g.coded_h, (x0 + px) * 4 + mvx, (y0 + py) * 4 + mvy);
            int d = abs(s - p);
            d = wave_sum(d);
            __syncthreads();
            if ((tid & 63) == 0) sub_cost[tid >> 6] = d;
            __syncthreads();
            cur_cost = me_cost(sub_cost[0] + sub_cost[1] + sub_cost[2] + sub_cost[3], lambda, mvx, mvy);
        }
        for (int step = 2; step >= 1; step >>= 1) {
            int bdx = 0, bdy = 0;
            uint32_t bcost = cur_cost;
            for (int k = 0; k < 8; ++k) {
                int ddx, ddy;
                subpel_offset(k, &ddx, &ddy);
                const int cx = mvx + ddx * step, cy = mvy + ddy * step;
                const int p = luma_qpel(ref, g.pitch, g.coded_w, g.coded_h, (x0 + px) * 4 + cx, (y0 + py) * 4 + cy);
                int d = wave_sum(abs(s - p));
                __syncthreads();
                if ((tid & 63) == 0) sub_cost[tid >> 6] = d;
                __syncthreads();
                const uint32_t cost = me_cost(sub_cost[0] + sub_cost[1] + sub_cost[2] + sub_cost[3], lambda, cx, cy);
                if (cost < bcost) {
                    bcost = cost;
                    bdx = ddx * step;
                    bdy = ddy * step;
                }
            }
            mvx += bdx;
            mvy += bdy;
            cur_cost = bcost;
        }
    }
    if (tid == 0) {
        mbs[mbi].mvx = (int16_t)mvx;
        mbs[mbi].mvy = (int16_t)mvy;
    }
}

// ------------------------------------------------------------------ inter encode
__global__ __launch_bounds__(256) void k_inter_encode(Geometry g, const FrameState* __restrict__ fs,
                                                       const uint8_t* __restrict__ src_y,
                                                       const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs,
                                                       int16_t* __restrict__ coef) {
    __shared__ uint8_t pred[4][384];
    __shared__ int16_t res[4][384];
    __shared__ int cdc[4][8];
    __shared__ int cdc_nz[4][2];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nmb = g.mb_w * g.mb_h;
    const int mbi = blockIdx.x * 4 + wave;
    const bool valid = mbi < nmb;
    const int mbx = valid ? mbi % g.mb_w : 0, mby = valid ? mbi / g.mb_w : 0;
    const int x0 = mbx * 16, y0 = mby * 16;
    const int qp = fs->qp;
    const int qpc = chroma_qp(qp, fs->chroma_qp_offset);
    const uint8_t* ref_y = fs->ref_y;
    const uint8_t* ref_uv = fs->ref_uv;
    const int cw = g.coded_w / 2, ch = g.coded_h / 2;
    int mvx = 0, mvy = 0;
    if (valid) {
        mvx = mbs[mbi].mvx;
        mvy = mbs[mbi].mvy;
        const int r = lane >> 2, c0 = (lane & 3) * 4;
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c0);
        for (int k = 0; k < 4; ++k) {
            const int p = luma_qpel(ref_y, g.pitch, g.coded_w, g.coded_h, (x0 + c0 + k) * 4 + mvx, (y0 + r) * 4 + mvy);
            pred[wave][r * 16 + c0 + k] = (uint8_t)p;
            res[wave][r * 16 + c0 + k] = (int16_t)((int)((sw >> (8 * k)) & 0xff) - p);
        }
        const int cr_ = lane >> 3, cc = lane & 7;
        const int xc = x0 / 2 + cc, yc = y0 / 2 + cr_;
        for (int comp = 0; comp < 2; ++comp) {
            const int p = chroma_pred8(ref_uv, g.pitch, cw, ch, comp, xc * 8 + mvx, yc * 8 + mvy);
            const int s = src_uv[yc * g.pitch + 2 * xc + comp];
            pred[wave][256 + comp * 64 + cr_ * 8 + cc] = (uint8_t)p;
            res[wave][256 + comp * 64 + cr_ * 8 + cc] = (int16_t)(s - p);
        }
    }
    __syncthreads();

    int z[16];
    int nz = 0;
    int16_t* mc = coef + (size_t)(valid ? mbi : 0) * kCoefStride;
    if (valid && lane < 16) {
        const int b = lane, bx = kBlkX[b], by = kBlkY[b];
        int x[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[wave][(by * 4 + i) * 16 + bx * 4 + j];
        int zs[16], r[16];
        nz = luma_block_inter(x, qp, zs, r);
        for (int k = 0; k < 16; ++k) mc[kCoefLuma + b * 16 + k] = (int16_t)zs[k];
        mbs[mbi].nz_luma[by * 4 + bx] = (uint8_t)nz;
        for (int i = 0; i < 4; ++i) {
            uint32_t packed = 0;
            for (int j = 0; j < 4; ++j) {
                const int v = clip255(pred[wave][(by * 4 + i) * 16 + bx * 4 + j] + r[i * 4 + j]);
                packed |= (uint32_t)v << (8 * j);
            }
            *reinterpret_cast<uint32_t*>(fs->rec_y + (y0 + by * 4 + i) * g.pitch + x0 + bx * 4) = packed;
        }
    } else if (valid && lane < 24) {
        const int comp = (lane - 16) >> 2, cb = (lane - 16) & 3, bx = cb & 1, by = cb >> 1;
        int x[16], y[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[wave][256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j];
        fdct4x4(x, y);
        cdc[wave][comp * 4 + cb] = y[0];
        nz = quant4x4(y, z, qpc, false, 1);
        for (int k = 1; k < 16; ++k) mc[kCoefChromaAc + (comp * 4 + cb) * 16 + k] = (int16_t)z[kZigzag4x4[k]];
        (comp ? mbs[mbi].nz_cr : mbs[mbi].nz_cb)[cb] = (uint8_t)nz;
    }
    __syncthreads();
    if (valid && (lane == 16 || lane == 20)) {
        const int comp = (lane - 16) >> 2;
        int in[4], zd[4], dq[4];
        for (int i = 0; i < 4; ++i) in[i] = cdc[wave][comp * 4 + i];
        const int n = quant_dc_chroma(in, zd, qpc, false);
        for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + comp * 4 + i] = (int16_t)zd[i];
        dequant_dc_chroma(zd, dq, qpc);
        for (int i = 0; i < 4; ++i) cdc[wave][comp * 4 + i] = dq[i];
        cdc_nz[wave][comp] = n;
    }
    __syncthreads();
    if (valid && lane >= 16 && lane < 24) {
        const int comp = (lane - 16) >> 2, cb = (lane - 16) & 3, bx = cb & 1, by = cb >> 1;
        int d[16], r[16];
        dequant4x4(z, d, qpc, 1);
        d[0] = cdc[wave][comp * 4 + cb];
        idct4x4(d, r);
        const int xc = x0 / 2 + bx * 4, yc = y0 / 2 + by * 4;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const int v = clip255(pred[wave][256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j] + r[i * 4 + j]);
                fs->rec_uv[(yc + i) * g.pitch + 2 * (xc + j) + comp] = (uint8_t)v;
            }
    }
    const unsigned long long luma_mask = __ballot(valid && lane < 16 && nz > 0);
    const unsigned long long chroma_mask = __ballot(valid && lane >= 16 && lane < 24 && nz > 0);
    if (valid && lane == 0) {
        int cbp = 0;
        for (int i8 = 0; i8 < 4; ++i8)
            if ((luma_mask >> (4 * i8)) & 0xf) cbp |= 1 << i8;
        const int cc = (chroma_mask != 0) ? 2 : ((cdc_nz[wave][0] | cdc_nz[wave][1]) ? 1 : 0);
        cbp |= cc << 4;
        MbInfo& m = mbs[mbi];
        m.type = kMbP16x16;
        m.cbp = (uint8_t)cbp;
        m.i16_mode = 0;
        m.chroma_mode = 0;
    }
}

// ------------------------------------------------------------------ intra (I slices)
// One wave per MB row; every row is its own slice, so the only neighbour is the left MB.
__global__ __launch_bounds__(64) void k_intra_rows(Geometry g, const FrameState* __restrict__ fs,
                                                    const uint8_t* __restrict__ src_y,
                                                    const uint8_t* __restrict__ src_uv, MbInfo* __restrict__ mbs,
                                                    int16_t* __restrict__ coef) {
    __shared__ uint8_t left[32];  // 16 luma, 8 cb, 8 cr: right column of the previous MB
    __shared__ uint8_t pred[384];
    __shared__ int16_t res[384];
    __shared__ int ldc[16];
    __shared__ int cdc[8];
    __shared__ int cdc_nz[2];
    __shared__ int modes[2];

    const int mby = blockIdx.x, lane = threadIdx.x;
    const int qp = fs->qp;
    const int qpc = chroma_qp(qp, fs->chroma_qp_offset);
    const int y0 = mby * 16;

    for (int mbx = 0; mbx < g.mb_w; ++mbx) {
        const int mbi = mby * g.mb_w + mbx, x0 = mbx * 16;
        const bool have_left = mbx > 0;
        // ---- mode decision (SAD) and prediction
        const int r = lane >> 2, c0 = (lane & 3) * 4;
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(src_y + (y0 + r) * g.pitch + x0 + c0);
        int dcl = 128;
        if (have_left) {
            int s = 0;
            for (int i = 0; i < 16; ++i) s += left[i];
            dcl = (s + 8) >> 4;
        }
        int sad_dc = 0, sad_h = 0;
        for (int k = 0; k < 4; ++k) {
            const int sv = (sw >> (8 * k)) & 0xff;
            sad_dc += abs(sv - dcl);
            sad_h += have_left ? abs(sv - left[r]) : 0;
        }
        sad_dc = wave_sum(sad_dc);
        sad_h = wave_sum(sad_h);
        const int lmode = (have_left && sad_h < sad_dc) ? 1 : 2;  // 1 = horizontal, 2 = DC
        for (int k = 0; k < 4; ++k) {
            const int sv = (sw >> (8 * k)) & 0xff;
            const int p = (lmode == 1) ? left[r] : dcl;
            pred[r * 16 + c0 + k] = (uint8_t)p;
            res[r * 16 + c0 + k] = (int16_t)(sv - p);
        }
        // chroma: DC (0) or horizontal (1); with no top neighbour DC uses the left column
        const int cr_ = lane >> 3, cc = lane & 7;
        const int xc = x0 / 2 + cc, yc = y0 / 2 + cr_;
        int sdc = 0, sh = 0;
        int pdc[2];
        for (int comp = 0; comp < 2; ++comp) {
            int d = 128;
            if (have_left) {
                const int rb = (cr_ >> 2) * 4;
                d = (left[16 + comp * 8 + rb] + left[16 + comp * 8 + rb + 1] + left[16 + comp * 8 + rb + 2] +
                     left[16 + comp * 8 + rb + 3] + 2) >> 2;
            }
            pdc[comp] = d;
            const int s = src_uv[yc * g.pitch + 2 * xc + comp];
            sdc += abs(s - d);
            sh += have_left ? abs(s - left[16 + comp * 8 + cr_]) : 0;
        }
        sdc = wave_sum(sdc);
        sh = wave_sum(sh);
        const int cmode = (have_left && sh < sdc) ? 1 : 0;
        for (int comp = 0; comp < 2; ++comp) {
            const int s = src_uv[yc * g.pitch + 2 * xc + comp];
            const int p = cmode == 1 ? left[16 + comp * 8 + cr_] : pdc[comp];
            pred[256 + comp * 64 + cr_ * 8 + cc] = (uint8_t)p;
            res[256 + comp * 64 + cr_ * 8 + cc] = (int16_t)(s - p);
        }
        __syncthreads();
        // ---- transform + quant
        int z[16];
        int nz = 0;
        int16_t* mc = coef + (size_t)mbi * kCoefStride;
        if (lane < 16) {
            const int b = lane, bx = kBlkX[b], by = kBlkY[b];
            int x[16], y[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[(by * 4 + i) * 16 + bx * 4 + j];
            fdct4x4(x, y);
            ldc[by * 4 + bx] = y[0];
            nz = quant4x4(y, z, qp, true, 1);
            for (int k = 1; k < 16; ++k) mc[kCoefLuma + b * 16 + k] = (int16_t)z[kZigzag4x4[k]];
            mc[kCoefLuma + b * 16] = 0;
        } else if (lane < 24) {
            const int comp = (lane - 16) >> 2, cb = (lane - 16) & 3, bx = cb & 1, by = cb >> 1;
            int x[16], y[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) x[i * 4 + j] = res[256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j];
            fdct4x4(x, y);
            cdc[comp * 4 + cb] = y[0];
            nz = quant4x4(y, z, qpc, true, 1);
            for (int k = 1; k < 16; ++k) mc[kCoefChromaAc + (comp * 4 + cb) * 16 + k] = (int16_t)z[kZigzag4x4[k]];
        }
        __syncthreads();
        if (lane == 0) {
            int zd[16], dq[16];
            quant_dc_luma(ldc, zd, qp);
            for (int k = 0; k < 16; ++k) mc[kCoefLumaDc + k] = (int16_t)zd[kZigzag4x4[k]];
            dequant_dc_luma(zd, dq, qp);
            for (int k = 0; k < 16; ++k) ldc[k] = dq[k];
        } else if (lane == 16 || lane == 20) {
            const int comp = (lane - 16) >> 2;
            int in[4], zd[4], dq[4];
            for (int i = 0; i < 4; ++i) in[i] = cdc[comp * 4 + i];
            const int n = quant_dc_chroma(in, zd, qpc, true);
            for (int i = 0; i < 4; ++i) mc[kCoefChromaDc + comp * 4 + i] = (int16_t)zd[i];
            dequant_dc_chroma(zd, dq, qpc);
            for (int i = 0; i < 4; ++i) cdc[comp * 4 + i] = dq[i];
            cdc_nz[comp] = n;
        }
        __syncthreads();
        const unsigned long long luma_mask = __ballot(lane < 16 && nz > 0);
        const unsigned long long chroma_mask = __ballot(lane >= 16 && lane < 24 && nz > 0);
        const bool luma_ac = luma_mask != 0;
        // ---- reconstruction
        if (lane < 16) {
            const int b = lane, bx = kBlkX[b], by = kBlkY[b];
            int d[16], rr[16];
            if (luma_ac) {
                dequant4x4(z, d, qp, 1);
            } else {
                for (int i = 1; i < 16; ++i) d[i] = 0;
            }
            d[0] = ldc[by * 4 + bx];
            idct4x4(d, rr);
            for (int i = 0; i < 4; ++i) {
                uint32_t packed = 0;
                for (int j = 0; j < 4; ++j) {
                    const int v = clip255(pred[(by * 4 + i) * 16 + bx * 4 + j] + rr[i * 4 + j]);
                    packed |= (uint32_t)v << (8 * j);
                    if (bx == 3 && j == 3) left[by * 4 + i] = (uint8_t)v;
                }
                *reinterpret_cast<uint32_t*>(fs->rec_y + (y0 + by * 4 + i) * g.pitch + x0 + bx * 4) = packed;
            }
            mbs[mbi].nz_luma[by * 4 + bx] = (uint8_t)(luma_ac ? nz : 0);
        } else if (lane < 24) {
            const int comp = (lane - 16) >> 2, cb = (lane - 16) & 3, bx = cb & 1, by = cb >> 1;
            int d[16], rr[16];
            dequant4x4(z, d, qpc, 1);
            d[0] = cdc[comp * 4 + cb];
            idct4x4(d, rr);
            const int xcb = x0 / 2 + bx * 4, ycb = y0 / 2 + by * 4;
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    const int v = clip255(pred[256 + comp * 64 + (by * 4 + i) * 8 + bx * 4 + j] + rr[i * 4 + j]);
                    fs->rec_uv[(ycb + i) * g.pitch + 2 * (xcb + j) + comp] = (uint8_t)v;
                    if (bx == 1 && j == 3) left[16 + comp * 8 + by * 4 + i] = (uint8_t)v;
                }
            (comp ? mbs[mbi].nz_cr : mbs[mbi].nz_cb)[cb] = (uint8_t)nz;
        }
        if (lane == 0) {
            const int ccbp = (chroma_mask != 0) ? 2 : ((cdc_nz[0] | cdc_nz[1]) ? 1 : 0);
            MbInfo& m = mbs[mbi];
            m.type = kMbI16x16;
            m.cbp = (uint8_t)((luma_ac ? 15 : 0) | (ccbp << 4));
            m.i16_mode = (uint8_t)lmode;
            m.chroma_mode = (uint8_t)cmode;
            m.mvx = 0;
            m.mvy = 0;
        }
        __syncthreads();
        (void)modes;
    }
}

// ------------------------------------------------------------------ CAVLC
__global__ __launch_bounds__(256) void k_cavlc(Geometry g, const FrameState* __restrict__ fs, MbInfo* __restrict__ mbs,
                                               const int16_t* __restrict__ coef, uint32_t* __restrict__ slot,
                                               uint32_t* __restrict__ slot_bits) {
    __shared__ uint32_t lds_slot[4][kSlotWords];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nmb = g.mb_w * g.mb_h;
    const int mbi = blockIdx.x * 4 + wave;
    for (int i = lane; i < kSlotWords; i += 64) lds_slot[wave][i] = 0;
    if (mbi >= nmb) return;  // whole wave exits together; no workgroup barrier below
    const int mbx = mbi % g.mb_w, mby = mbi / g.mb_w;
    const Avail av = mb_avail(g, mbx, mby, fs->slice_rows);
    const MbInfo m = mbs[mbi];
    const int16_t* mc = coef + (size_t)mbi * kCoefStride;

    // motion vector prediction + P_Skip decision (every lane computes the same values)
    int mvdx = 0, mvdy = 0;
    const bool skip = decide_skip(g, mbs, mbi, av, &mvdx, &mvdy);
    uint32_t bits = 0;
    if (!skip && lane < kNumRoles) {
        BitCounter bc;
        bc.init(nullptr);
        code_role(bc, lane, g, fs->idr, mbs, m, mc, mbi, av, mvdx, mvdy);
        bits = bc.bits;
    }
    // exclusive prefix sum of bits over lanes
    uint32_t incl = bits;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    const uint32_t off = incl - bits;
    __builtin_amdgcn_wave_barrier();
    if (!skip && lane < kNumRoles && bits > 0 && total <= kSlotWords * 32u) {
        OrWriter<false> w;
        w.init(lds_slot[wave], off);
        code_role(w, lane, g, fs->idr, mbs, m, mc, mbi, av, mvdx, mvdy);
        w.flush();
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t nwords = (total + 31) >> 5;
    for (uint32_t i = lane; i < nwords && i < (uint32_t)kSlotWords; i += 64)
        slot[(size_t)mbi * kSlotWords + i] = lds_slot[wave][i];
    if (lane == 0) {
        slot_bits[mbi] = total <= kSlotWords * 32u ? total : 0xffffffffu;
        mbs[mbi].skip = skip ? 1 : 0;
    }
}

// ------------------------------------------------------------------ scan
constexpr int kScanThreads = 1024;

__device__ __forceinline__ SliceParams slice_params(const FrameState* fs, int s, int mb_w) {
    return make_slice_params(s * fs->slice_rows * mb_w, fs->idr, fs->frame_num, fs->log2_max_frame_num,
                             fs->idr_pic_id, fs->qp - fs->pic_init_qp, fs->deblock_off);
}

__global__ __launch_bounds__(kScanThreads) void k_scan(Geometry g, const FrameState* __restrict__ fs,
                                                       const MbInfo* __restrict__ mbs,
                                                       const uint32_t* __restrict__ slot_bits,
                                                       uint32_t* __restrict__ unit_off, int32_t* __restrict__ skip_run,
                                                       uint32_t* __restrict__ slice_info, uint32_t* __restrict__ out,
                                                       size_t out_words, OutHeader* __restrict__ hdr) {
    __shared__ int s_i[kScanThreads];
    __shared__ uint32_t s_u[kScanThreads];
    __shared__ uint32_t s_overflow;
    const int t = threadIdx.x;
    const int nmb = g.mb_w * g.mb_h;
    const int rows = fs->slice_rows;
    const int ns = fs->num_slices;
    const int per_slice = rows * g.mb_w;
    const int C = (nmb + kScanThreads - 1) / kScanThreads;
    const int lo = t * C, hi = min(lo + C, nmb);
    if (t == 0) s_overflow = 0;

    // 1. last coded (non-skipped) MB per chunk -> exclusive max scan
    int last = -1;
    for (int i = lo; i < hi; ++i)
        if (!mbs[i].skip) last = i;
    s_i[t] = last;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        int v = t >= o ? s_i[t - o] : -1;
        __syncthreads();
        s_i[t] = max(s_i[t], v);
        __syncthreads();
    }
    int carry = t > 0 ? s_i[t - 1] : -1;
    __syncthreads();
    // 2. skip runs and unit bit lengths; local sums
    uint32_t local = 0;
    for (int i = lo; i < hi; ++i) {
        const int s = i / per_slice;
        const int first = s * per_slice;
        const int prev = max(carry, first - 1);
        const bool coded = !mbs[i].skip;
        uint32_t ub = 0;
        if (coded) {
            const int run = i - prev - 1;
            skip_run[i] = run;
            uint32_t sb = slot_bits[i];
            if (sb == 0xffffffffu) {
                s_overflow = 1;
                sb = 0;
            }
            ub = (fs->idr ? 0 : ue_len((uint32_t)run)) + sb;
            carry = i;
        } else {
            skip_run[i] = -1;
        }
        const int slast = min(first + per_slice, nmb) - 1;
        if (i == slast) slice_info[4 * s + 3] = coded ? 0u : (uint32_t)(i - prev);
        unit_off[i] = ub;  // temporarily: unit bits
        local += ub;
    }
    s_u[t] = local;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        uint32_t v = t >= o ? s_u[t - o] : 0;
        __syncthreads();
        s_u[t] += v;
        __syncthreads();
    }
    uint32_t run_sum = t > 0 ? s_u[t - 1] : 0;
    for (int i = lo; i < hi; ++i) {  // unit_off <- exclusive global prefix (E[i])
        const uint32_t ub = unit_off[i];
        unit_off[i] = run_sum;
        run_sum += ub;
    }
    const uint32_t grand_total = s_u[kScanThreads - 1];
    __syncthreads();
    // 3. per slice sizes (one thread per slice; ns <= kMaxSlices <= kScanThreads)
    uint32_t sbytes = 0;
    uint32_t ebase = 0, hbits = 0;
    if (t < ns) {
        const int first = t * per_slice;
        const int slast = min(first + per_slice, nmb) - 1;
        ebase = unit_off[first];
        const uint32_t eend = (slast + 1 < nmb) ? unit_off[slast + 1] : grand_total;
        BitCounter bc;
        bc.init(nullptr);
        write_slice_header(bc, slice_params(fs, t, g.mb_w));
        hbits = bc.bits;
        const uint32_t trail = fs->idr ? 0u : slice_info[4 * t + 3];
        const uint32_t bits = hbits + (eend - ebase) + (trail ? ue_len(trail) : 0) + 1;
        sbytes = (bits + 7) >> 3;
    }
    __syncthreads();
    s_u[t] = sbytes;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {
        uint32_t v = t >= o ? s_u[t - o] : 0;
        __syncthreads();
        s_u[t] += v;
        __syncthreads();
    }
    const uint32_t total_bytes = s_u[kScanThreads - 1];
    if (t < ns) {
        slice_info[4 * t + 0] = hbits;
        slice_info[4 * t + 1] = s_u[t] - sbytes;  // byte offset
        slice_info[4 * t + 2] = sbytes;
        s_i[t] = (int)ebase;
    }
    __syncthreads();
    // 4. absolute unit offsets
    for (int i = lo; i < hi; ++i) {
        const int s = i / per_slice;
        unit_off[i] = slice_info[4 * s + 1] * 8 + slice_info[4 * s + 0] + (unit_off[i] - (uint32_t)s_i[s]);
    }
    // 5. zero the payload words that k_pack will OR into
    const size_t nwords = ((size_t)total_bytes + 3) / 4;
    const bool over = nwords > out_words;
    for (size_t i = t; i < nwords && i < out_words; i += kScanThreads) out[i] = 0;
    __syncthreads();
    if (t == 0) {
        hdr->total_bytes = over ? 0 : total_bytes;
        hdr->num_slices = ns;
        hdr->overflow = s_overflow | (over ? 2u : 0u);
    }
}

// ------------------------------------------------------------------ pack
__global__ __launch_bounds__(256) void k_pack(Geometry g, const FrameState* __restrict__ fs,
                                              const MbInfo* __restrict__ mbs, const uint32_t* __restrict__ slot,
                                              const uint32_t* __restrict__ slot_bits,
                                              const uint32_t* __restrict__ unit_off,
                                              const int32_t* __restrict__ skip_run,
                                              const uint32_t* __restrict__ slice_info, uint32_t* __restrict__ out,
                                              const OutHeader* __restrict__ hdr) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nmb = g.mb_w * g.mb_h;
    const int u = blockIdx.x * 4 + wave;
    if (hdr->overflow) return;
    if (u < nmb) {
        const int run = skip_run[u];
        if (run < 0) return;
        uint32_t pos = unit_off[u];
        if (!fs->idr) {
            if (lane == 0) {
                OrWriter<true> w;
                w.init(out, pos);
                put_ue(w, (uint32_t)run);
                w.flush();
            }
            pos += ue_len((uint32_t)run);
        }
        const uint32_t nb = slot_bits[u];
        const uint32_t nw = (nb + 31) >> 5;
        const uint32_t* src = slot + (size_t)u * kSlotWords;
        for (uint32_t i = lane; i < nw; i += 64) {
            const uint32_t v = src[i];
            const int n = (i == nw - 1) ? (int)(nb - 32 * i) : 32;
            OrWriter<true> w;
            w.init(out, pos + 32 * i);
            w.emit(v, n);
        }
        return;
    }
    const int s = u - nmb;
    if (s >= fs->num_slices || lane != 0) return;
    const uint32_t hbits = slice_info[4 * s + 0];
    const uint32_t byte_off = slice_info[4 * s + 1];
    const uint32_t bytes = slice_info[4 * s + 2];
    OrWriter<true> w;
    w.init(out, byte_off * 8);
    write_slice_header(w, slice_params(fs, s, g.mb_w));
    w.flush();
    // trailer: optional trailing mb_skip_run, then rbsp_stop_one_bit at the end of data
    const int per_slice = fs->slice_rows * g.mb_w;
    const int first = s * per_slice, slast = min(first + per_slice, nmb) - 1;
    // find end of data: the last coded MB's unit end, or header end if none
    const uint32_t trail = fs->idr ? 0u : slice_info[4 * s + 3];
    uint32_t data_end = byte_off * 8 + hbits;
    for (int i = slast; i >= first; --i) {
        if (skip_run[i] >= 0) {
            data_end = unit_off[i] + (fs->idr ? 0 : ue_len((uint32_t)skip_run[i])) + slot_bits[i];
            break;
        }
    }
    OrWriter<true> t2;
    t2.init(out, data_end);
    if (trail) put_ue(t2, trail);
    t2.put(1, 1);
    t2.flush();
    (void)bytes;
}

// ------------------------------------------------------------------ copy to host
__global__ __launch_bounds__(256) void k_copy_out(const uint32_t* __restrict__ out, const OutHeader* __restrict__ hdr,
                                                  const uint32_t* __restrict__ slice_info, uint8_t* __restrict__ host) {
    const uint32_t total = hdr->total_bytes;
    const uint32_t ns = hdr->num_slices;
    const size_t gid = blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    if (gid == 0) *reinterpret_cast<OutHeader*>(host) = *hdr;
    uint32_t* hs = reinterpret_cast<uint32_t*>(host + sizeof(OutHeader));
    for (size_t s = gid; s < ns; s += stride) {
        hs[s] = slice_info[4 * s + 1];
        hs[kMaxSlices + s] = slice_info[4 * s + 2];
    }
    const size_t n16 = ((size_t)total + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(out);
    uint4* dst = reinterpret_cast<uint4*>(host + kOutPayloadOffset);
    for (size_t i = gid; i < n16; i += stride) dst[i] = src[i];
}

}  // namespace

void launch_me(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, hipStream_t stream) {
    const int nmb = g.mb_w * g.mb_h;
    hipLaunchKernelGGL(k_me_full, dim3(nmb), dim3(256), 0, stream, g, b.fs, src_y, b.mb);
}

void launch_inter(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream) {
    const int nmb = g.mb_w * g.mb_h;
    hipLaunchKernelGGL(k_inter_encode, dim3((nmb + 3) / 4), dim3(256), 0, stream, g, b.fs, src_y, src_uv, b.mb,
                       b.coef);
}

void launch_intra(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream) {
    hipLaunchKernelGGL(k_intra_rows, dim3(g.mb_h), dim3(64), 0, stream, g, b.fs, src_y, src_uv, b.mb, b.coef);
}

void launch_entropy(const Geometry& g, const DeviceBuffers& b, uint8_t* host_out, hipStream_t stream) {
    const int nmb = g.mb_w * g.mb_h;
    hipLaunchKernelGGL(k_cavlc, dim3((nmb + 3) / 4), dim3(256), 0, stream, g, b.fs, b.mb, b.coef, b.slot,
                       b.slot_bits);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(kScanThreads), 0, stream, g, b.fs, b.mb, b.slot_bits, b.unit_off,
                       b.skip_run, b.slice_info, b.out, b.out_words, b.out_hdr);
    const int units = nmb + g.mb_h;  // MBs + at most mb_h slices
    hipLaunchKernelGGL(k_pack, dim3((units + 3) / 4), dim3(256), 0, stream, g, b.fs, b.mb, b.slot, b.slot_bits,
                       b.unit_off, b.skip_run, b.slice_info, b.out, b.out_hdr);
    hipLaunchKernelGGL(k_copy_out, dim3(128), dim3(256), 0, stream, b.out, b.out_hdr, b.slice_info, host_out);
}

}  // namespace h264
}  // namespace mx
