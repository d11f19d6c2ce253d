// Device data layout and host API of the HIP H.264 encoder.
//
// Per-frame kernel chain (all on one HIP stream, graph-capturable):
//   P frame: k_hpel -> k_me_full -> k_inter_encode -> k_intra_analyze -> k_intra_wave
//            -> k_cavlc -> k_scan -> k_pack
//   I frame: k_intra_analyze -> k_intra_wave -> k_cavlc -> k_scan -> k_pack
// k_intra_analyze decides every macroblock's intra modes open-loop (SATD against predictions
// from source neighbours, fully parallel); k_intra_wave reconstructs the intra macroblocks
// closed-loop in a diagonal wavefront (one luma and one chroma wave per MB row).
// k_pack writes the payload straight into pinned host memory (zero-copy).
// Only the slice payloads (RBSP, byte aligned) leave the GPU; the host adds start
// codes, NAL headers and emulation-prevention bytes (h264_encoder.cpp).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXHD_GPU __host__ __device__ __forceinline__

namespace mx {
namespace h264 {

constexpr int kSlotWords = 640;   // per-MB CAVLC bit slot (2560 B >= worst case)
constexpr int kCoefStride = 416;  // int16 coefficients per MB
constexpr int kCoefLuma = 0;      // [16 blkIdx][16 scan]
constexpr int kCoefLumaDc = 256;  // [16 scan]
constexpr int kCoefChromaDc = 272;  // [2][4]
constexpr int kCoefChromaAc = 280;  // [2][4 blk][16 scan], index 0 unused

enum MbType : uint8_t { kMbP16x16 = 0, kMbI16x16 = 1, kMbI4x4 = 2 };

struct MbInfo {
    int16_t mvx, mvy;  // quarter-pel
    uint8_t type;      // MbType
    uint8_t cbp;       // bits 0..3 luma 8x8, bits 4..5 chroma (0/1/2)
    uint8_t i16_mode;  // Intra16x16 prediction mode
    uint8_t chroma_mode;
    uint8_t nz_luma[16];  // TotalCoeff per 4x4 block, raster (by*4+bx)
    uint8_t nz_cb[4];     // chroma AC TotalCoeff, raster 2x2
    uint8_t nz_cr[4];
    uint8_t skip;  // set by k_cavlc
    uint8_t qp;    // macroblock QP (frame QP + adaptive-quantisation offset)
    uint8_t cbp_c; // chroma cbp of an intra MB, written by the chroma wave of k_intra_wave / k_intra_p
    uint8_t itype; // P pictures: the intra type k_intra_analyze decided (applied if k_intra_p selects the MB)
    uint8_t i4[8];     // Intra4x4 prediction modes, two per byte, raster block order
    uint32_t cost;     // P pictures: inter luma SATD cost (+ mv rate), for the intra decision
    // inter partitioning (H.264 P pictures): part 0 = P_L0_16x16 (vector mvx / mvy), 1 = 16x8,
    // 2 = 8x16 with the vectors of partitions 0 / 1 in pmv[0..1] / pmv[2..3] (quarter-pel).
    // mvx / mvy always keep the best 16x16 vector (the HEVC and VP8 encoders read only those).
    int16_t pmv[4];
    uint8_t part;
    uint8_t pad_[7];
};
static_assert(sizeof(MbInfo) == 64, "MbInfo layout");
enum MbPart : uint8_t { kPart16x16 = 0, kPart16x8 = 1, kPart8x16 = 2 };

MXHD_GPU bool is_intra(const MbInfo& m) { return m.type != kMbP16x16; }
// Whether macroblock (mbx, mby) is outside the quality-report mask of the frame state.
template <class FS>
MXHD_GPU bool mb_unmasked(const FS* fs, int mbx, int mby) {
    return !(mbx >= fs->mask_mx0 && mbx < fs->mask_mx1 && mby >= fs->mask_my0 && mby < fs->mask_my1);
}
// mb_qp_delta present: Intra16x16 always, other macroblocks when they carry residual.
MXHD_GPU bool carries_dqp(const MbInfo& m) { return m.type == kMbI16x16 || m.cbp != 0; }

// Per-frame state, written by the host into pinned memory and copied to the device at
// the start of every frame (one memcpy node), so a captured graph replays correctly.
struct FrameState {
    const uint8_t* ref_y;
    const uint8_t* ref_uv;
    uint8_t* rec_y;
    uint8_t* rec_uv;
    int32_t idr;
    int32_t frame_num;
    int32_t idr_pic_id;
    int32_t qp;
    int32_t slice_rows;  // MB rows per slice
    int32_t num_slices;
    int32_t search_range;  // integer-pel full-search radius
    int32_t subpel;        // 1 = quarter-pel refinement
    int32_t me_coarse;     // 1 = even-offset grid + integer neighbours instead of the full search
    int32_t intra4x4;      // 0 = intra MBs are Intra16x16 only
    int32_t deblock_off;   // disable_deblocking_filter_idc (0: k_deblock filters the reconstruction)
    int32_t db_epoch;      // nonzero, new every frame: tag of k_deblock's cross-workgroup hand-off words
    int32_t pic_init_qp;
    int32_t chroma_qp_offset;
    int32_t log2_max_frame_num;
    int32_t hp_pitch;  // pitch of the padded half-pel planes
    int32_t aq;        // adaptive quantisation on/off (P frames)
    int32_t intra_in_p;  // P frames: k_intra_analyze / k_intra_wave run (distortion deltas included)
    int32_t partitions;  // P frames: k_me_full also searches 16x8 / 8x16 partitionings (H.264)
    // quality report: MBs in [mask_mx0, mask_mx1) x [mask_my0, mask_my1) are left out of the 4th
    // distortion channel (e.g. the synthetic desktop's noise panel); empty rect = no mask
    int32_t mask_mx0, mask_my0, mask_mx1, mask_my1;
    // temporal AQ classes (aq 3): previous frame's source luma (read) and this frame's copy (written
    // by k_inter_encode per MB, by a copy for IDR pictures); coded size, luma pitch
    const uint8_t* prev_src;
    uint8_t* save_src;
    // padded reference planes (origin at picture (0,0), valid for x,y in [-kHpelPad, size+kHpelPad))
    const uint8_t* hp_f;  // full-sample (edge-replicated)
    const uint8_t* hp_h;  // horizontal half sample b at (x+1/2, y)
    const uint8_t* hp_v;  // vertical half sample h at (x, y+1/2)
    const uint8_t* hp_j;  // centre half sample j at (x+1/2, y+1/2)
    // motion-search planes (k_me_full): the padded F / H / V / J planes of the reference picture's
    // reconstruction BEFORE its in-loop filter when that picture was deblocked -- the next
    // picture's search then depends only on the reconstruction, not on the filter, and runs beside
    // it on another stream (profiles/r06_deblock) -- nullptr: the hp_* planes
    const uint8_t* me_f;
    const uint8_t* me_h;
    const uint8_t* me_v;
    const uint8_t* me_j;
    // distortion partials (Y, U, V, Y outside the mask MBs) over the display area, [4][kSsePartStride]: one per
    // inter workgroup / intra MB row, reduced by k_scan into OutHeader (no atomics)
    unsigned long long* sse_part;
};
constexpr int kHpelPad = 48;
constexpr int kSsePartStride = 65536;  // >= ceil(nmb / 4): 8K is 129600 MBs -> 32400 partials

// Header written at the start of the device output / host output buffer.
struct OutHeader {
    uint32_t total_bytes;  // payload bytes (all slices, byte aligned)
    uint32_t num_slices;
    uint32_t overflow;     // nonzero if any MB exceeded its slot
    uint32_t deblocked;    // the picture's disable_deblocking_filter_idc was 0
    uint64_t sse[3];      // source vs reconstruction squared error (Y, U, V)
    uint64_t sse_masked;   // Y outside the mask macroblocks (FrameState::mask_*)
    // device wall clock (hipDeviceAttributeWallClockRate): start of the frame's first encoder kernel,
    // end of its last (k_pack) -- per-frame GPU time without timing events on the streams (an
    // event record between kernels cost ~5 us of idle GPU each: profiles/r04_h264)
    uint64_t t_start;
    uint64_t t_end;
    // adaptive filter (EncoderConfig::deblock 2): the P picture's class counts (h264_deblock.h
    // db_auto_count, k_scan_rows), from which the host decides the next picture's filter
    uint32_t db_coherent, db_changed, db_moving;
    uint32_t pad;
};
static_assert(sizeof(OutHeader) % 16 == 0, "payload must stay 16-byte aligned");
constexpr int kMaxSlices = 1024;
// slice_info fields: 0 header bits, 1 byte offset, 2 bytes, 3 trailing skip run,
// 4 data-end bit (trailer start), 5 unit-bit prefix at the slice's first MB,
// 6 / 7 first / end rank of the slice's coded MBs in coded_info
constexpr int kSliceInfo = 8;
// host buffer: OutHeader | uint32 slice_off[kMaxSlices] | uint32 slice_len[kMaxSlices] | payload
constexpr size_t kOutPayloadOffset = sizeof(OutHeader) + 2 * kMaxSlices * sizeof(uint32_t);

struct Geometry {
    int width, height;  // display size
    int mb_w, mb_h;
    int pitch;          // luma pitch (bytes); UV plane has the same pitch
    int coded_w, coded_h;  // mb_w*16, mb_h*16
};

// Device buffers owned by the GPU encoder.
struct DeviceBuffers {
    FrameState* fs;         // device copy of the frame state
    MbInfo* mb;             // [nmb]
    int16_t* coef;          // [nmb * kCoefStride]
    uint32_t* slot;         // [nmb * kSlotWords]
    uint32_t* slot_bits;    // [nmb]
    uint4* row_agg;         // [mb_h] per MB row: first / last coded MB, coded count | overflow, unit bits
    unsigned long long* row_sse;  // [4][512] per-row distortion sums (k_scan_rows)
    uint4* coded_info;      // [nmb] per coded rank: {absolute bit offset, MB index, unit bits, skip run}
    uint32_t* quad_unit;    // [out_bytes / 16] per 128-bit output quad: rank of the unit holding its first bit
    uint32_t* slice_info;   // [kSliceInfo * kMaxSlices]
    size_t out_bytes;       // payload capacity of the host output buffer
    OutHeader* out_hdr;     // device header
    unsigned long long* sse_part;       // [4 * kSsePartStride] distortion partials
    int* wave_prog;         // [1] intra candidate count of P pictures ([0] unused)
    int32_t* intra_gain;    // [nmb] P frames: gain of switching each MB to intra (0 = stays inter)
    int* intra_cand;        // [nmb] P frames: MBs with a positive gain (count in wave_prog[1])
    uint32_t* mb_sse;       // [3 * nmb] P frames: per-MB inter distortion (replaced for intra MBs)
    // in-loop deblocking (h264_deblock.hip)
    uint4* db_rec;          // [nmb] boundary strengths + QP record per MB (k_db_prep)
    int* db_rowq;           // [mb_h] QP of each row's last mb_qp_delta MB (-1: none)
    uint64_t* db_glb;       // [2][mb_h][mb_w][24] band-boundary hand-off words (epoch-tagged, k_deblock)
    int* db_err;            // mapped host word: nonzero if a deblocking spin timed out
    uint32_t* db_cnt;       // [3] adaptive filter: coherent / changed / moving counts (k_scan_rows, zeroed by k_scan_out)
    uint32_t* pack_done;    // [1] k_pack workgroups finished (the last one stamps t_end and resets it)
};

// Kernel launchers (h264_kernels.hip).  All enqueue on `stream`; no host sync.
// state: the frame state by value (the search runs on a side stream before the analysis stream's
// first kernel has published it), or nullptr to read the published copy
void launch_me(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, hipStream_t stream,
               const FrameState* state = nullptr);
// F / H / V / J planes of an explicit luma picture (the unfiltered reconstruction of a picture the
// in-loop filter is about to modify), for the next picture's motion search (FrameState::me_*)
void launch_hpel_of(const Geometry& g, const uint8_t* luma, uint8_t* const planes[4], int hp_pitch, hipStream_t stream);
void launch_inter(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream);
// The first kernel of a frame (launch_intra for I, launch_hpel for P) publishes the frame
// state: with `publish` non-null it takes the state by value and stores it to b.fs for the
// later kernels (no copy node); with nullptr it reads b.fs (filled by a memcpy node, hipGraph).
void launch_intra(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                  hipStream_t stream, const FrameState* publish = nullptr);
// Build the padded F/H/V/J planes of the reference luma (b.fs->ref_y) into `planes` (4 planes,
// each hp_pitch x (coded_h + 2*kHpelPad), origin offset applied by the caller via FrameState).
void launch_hpel(const Geometry& g, const DeviceBuffers& b, uint8_t* const planes[4], int hp_pitch,
                 hipStream_t stream, const FrameState* publish = nullptr);
// In-loop deblocking of the reconstruction (FrameState::rec_y / rec_uv, in place) + the distortion
// partials of the filtered picture (h264_deblock.hip); after the analysis kernels.
// diagnostics: device wall-clock (start, end) of every row wave of the last k_deblock, luma rows
// then chroma rows
std::vector<unsigned long long> deblock_row_stamps(int mb_h);
void launch_deblock(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                    hipStream_t stream);
// Copy the source luma into FrameState::save_src (IDR pictures; the pointer is read on the device
// so a captured graph stays valid while the buffers alternate).
void launch_save_src(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, hipStream_t stream);
// wait_for_sse: event the stream waits on after k_cavlc, before the distortion partials are
// reduced (the deblocking kernels' completion on the analysis stream), or nullptr
void launch_entropy(const Geometry& g, const DeviceBuffers& b, uint8_t* host_out, hipStream_t stream,
                    hipEvent_t wait_for_sse = nullptr);
// P pictures, after launch_inter: open-loop intra analysis of every MB (intra vs inter) and the
// closed-loop reconstruction of the MBs that switched to intra.
void launch_intra_in_p(const Geometry& g, const DeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                       hipStream_t stream);

}  // namespace h264
}  // namespace mx
