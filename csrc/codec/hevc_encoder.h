// Host-side HEVC encoder API: GpuHevcEncoder (HIP kernels, production path) and
// CpuHevcEncoder (same decisions and syntax, serial C++ over the shared hevc_core.h
// functions; bit-exact oracle of the GPU encoder in tests).
//
// Reference parity: the reference's WEBRTC_ENCODER selects a GStreamer encoder element
// (reference Dockerfile:210, README.md:21); the HEVC configuration of BASELINE.json ("4K60
// HEVC, HIP CSC+scale path") runs through these classes ("mxh265enc").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <array>
#include <deque>
#include <vector>

#include "h264_encoder.h"
#include "hevc_core.h"

namespace mx {
namespace hevc {

using h264::EncoderConfig;
using h264::FrameStats;
using h264::Geometry;

// Level (A.4) for a picture size / frame rate, as general_level_idc (30 x level).
int pick_level(int width, int height, int fps);
int max_slices_for_level(int level_idc);

// Parameter sets, slice headers and Annex-B assembly shared by both encoders.  Rate
// control and IDR scheduling come from h264::EncoderCommon (codec independent).
class HevcCommon {
   public:
    explicit HevcCommon(const EncoderConfig& c);
    h264::EncoderCommon& rc() { return rc_; }
    const h264::EncoderCommon& rc() const { return rc_; }
    const EncoderConfig& config() const { return rc_.config(); }
    // 16x16 analysis units (the encoder's CU grid; historical names) and the 32x32 CTB grid
    int ctb_w() const { return rc_.mb_w(); }
    int ctb_h() const { return rc_.mb_h(); }
    int c32_w() const { return ctb_cols(ctb_w()); }
    int c32_h() const { return ctb_rows(ctb_h()); }
    int num_ctbs() const { return c32_w() * c32_h(); }
    // max_transform_hierarchy_depth_inter: 3 with split inter transform trees (a CU32's 16x16
    // quadrants at depth 1 may split too), else 0
    int depth_inter() const { return config().tu_split ? 3 : 0; }
    // max_transform_hierarchy_depth_intra: 1 when intra CU16s may split into four 8x8 luma / 4x4 chroma
    // TUs (EncoderConfig::hevc_intra_split), else 0
    int depth_intra() const { return config().hevc_intra_split ? 1 : 0; }
    int slice_rows() const { return slice_rows_; }  // CTB rows per I slice
    int i_split() const { return i_split_; }        // I slices per CTB row (segments)
    int i_seg_w() const { return 2 * ((c32_w() + i_split_ - 1) / i_split_); }  // 16x16-unit columns per segment
    int num_slices() const { return (c32_h() + slice_rows_ - 1) / slice_rows_ * i_split_; }
    int level_idc() const { return level_; }
    int max_slices() const { return max_slices_; }  // level limit (MaxSliceSegmentsPerPicture), capped
    // POC LSB (8 bits) of the current frame = frames since the last IDR.
    int poc() const { return rc_.cur_frame_num(); }
    void write_parameter_sets(std::vector<uint8_t>& out) const;
    // One slice segment NAL (slice starting at CTB `addr`): start code, NAL header, header +
    // payload with emulation prevention.  WPP: data holds the slice's substreams back to back,
    // sub_len[0..nsub) their raw sizes; the header carries their entry points (sizes after
    // emulation prevention, 7.4.7.1).
    // sub_off: byte offsets of the substreams in data (nullptr: back to back).
    // deblock: the picture's filter decision (adaptive filtering overrides the PPS per slice)
    void write_slice_nal(std::vector<uint8_t>& out, int addr, bool idr, int poc, int qp, bool deblock,
                         const uint8_t* data, size_t n, const uint32_t* sub_len = nullptr, int nsub = 0,
                         const uint32_t* sub_off = nullptr) const;
    bool wpp() const { return config().hevc_wpp != 0; }
    // CTB rows per P slice with WPP (the whole picture when 0 or larger)
    int wpp_rows() const {
        const int r = config().hevc_wpp_rows;
        return (r <= 0 || r > c32_h()) ? c32_h() : std::max(r, slice_rows_);  // level slice cap
    }
    // Slice layout: I pictures one slice per slice_rows() CTB rows (the intra wavefront needs a
    // fixed layout), P pictures cost-balanced raster runs of CTBs (plan_p_slices).  Returns first CTBs.
    std::vector<int> row_slices() const;
    std::vector<int> plan_p_slices(const std::vector<CuInfo>& cus) const;

   private:
    h264::EncoderCommon rc_;
    int slice_rows_ = 1;
    int i_split_ = 1;
    int level_ = 0;
    int max_slices_ = 1;
};

// Open-loop intra mode of a 16x16 unit (hevc_cpu.cpp; the GPU's k_hevc_intra_modes), with
// kIntraSplitFlag set when split (nonzero safe_split) codes it as four 8x8 TUs.
int intra_decide_mode(const uint8_t* sy, int pitch, int mb_w, int mb_h, int x, int y, int sr, int seg_w, int qp,
                      uint64_t safe, uint64_t safe_split = 0, bool split = false);
// Direct vs bin-token CABAC on random slices (hevc_cpu.cpp); returns the slices checked.
int token_selftest(uint32_t seed, int slices);
// Entropy-code the slice of CTBs [first, end) with wavefront parallel processing (host): every CTB
// row of the slice is a substream (fresh contexts in the slice's first row -- or when the picture
// is one CTB wide -- else the contexts the row above had after its second CTB), written to `out` back to back;
// sub_len receives one size per row.  Returns the total bytes.
uint32_t code_slice_wpp(uint8_t* out, uint32_t cap, bool islice, int slice_qp, const PicSyn& ps, int first, int end,
                        uint16_t* tok, std::vector<uint32_t>& sub_len);

class CpuHevcEncoder {
   public:
    explicit CpuHevcEncoder(const EncoderConfig& cfg);
    // NV12 frame in host memory (pitch shared by both planes, at least the coded size readable;
    // h264::pad_nv12 pads display-sized frames).
    const std::vector<uint8_t>& encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr = false);
    const FrameStats& last_stats() const { return stats_; }
    HevcCommon& common() { return common_; }
    const std::vector<uint8_t>& recon_y() const { return rec_y_[cur_]; }
    const std::vector<uint8_t>& recon_uv() const { return rec_uv_[cur_]; }
    int coded_pitch() const { return cw_; }
    const std::vector<CuInfo>& cus() const { return cu_; }

   private:
    void analyse_intra(const uint8_t* y, const uint8_t* uv, int pitch);
    void analyse_inter(const uint8_t* y, const uint8_t* uv, int pitch);
    int frame_qp_() { return qp_override_ >= 0 ? qp_override_ : common_.rc().cur_qp(); }
    int qp_override_ = -1;  // rate-control probe of the first picture
    // the picture's in-loop filter decision (EncoderConfig::deblock; adaptive: as k_hevc_db_auto)
    bool deblock_now_ = false, db_prev_on_ = false;

    EncoderConfig cfg_;
    HevcCommon common_;
    int cw_, ch_;
    std::vector<uint8_t> rec_y_[2], rec_uv_[2];
    int cur_ = 0;
    bool have_ref_ = false;
    std::vector<CuInfo> cu_;
    std::vector<int16_t> mv_;  // per CU (x, y)
    std::vector<int> slices_;  // first CTB of every slice of the current picture
    std::vector<uint8_t> qp_pred_, qpy_;  // per unit: QP predictor / QpY (slice_qp_chain)
    uint64_t bl_safe_ = 0;     // intra modes safe with a pending below-left (bl_safe_modes, luma 16 & chroma 8)
    uint64_t bl_safe_split_ = 0;  // ... of a split unit (bl_safe_split: luma 8 & chroma 4)
    std::vector<int16_t> coef_;
    std::vector<uint8_t> au_;
    std::vector<uint8_t> prev_src_;  // previous source luma (coded size), temporal AQ classes
    std::vector<uint32_t> sao_;      // SAO parameters, 4 words per CTB32 (hevc_core.h sao_pack)
    std::vector<uint16_t> tok_ = std::vector<uint16_t>(kMaxCuTokens);  // bin tokens of one CTU
    FrameStats stats_;
};

// ---------------------------------------------------------------- GPU encoder
// Per-frame kernel chain (hevc_kernels.hip):
//   P: k_hpel -> k_me_full (shared with H.264) -> k_hevc_inter
//   I: k_hevc_intra (one workgroup per slice, wavefront over its CTU rows)
//   then k_hevc_layout (slices: rows for I, cost-balanced runs for P) -> k_hevc_decide (P:
//   skip/merge/AMVP per slice) -> k_hevc_cabac (one wave per slice) -> k_hevc_pack
struct HevcFrameState {
    const uint8_t* ref_y;
    const uint8_t* ref_uv;
    uint8_t* rec_y;
    uint8_t* rec_uv;
    const uint8_t* hp_f;  // padded full-sample reference luma (origin at picture (0,0))
    int32_t hp_pitch;
    int32_t idr;
    int32_t qp;
    int32_t slice_rows;  // 16x16-unit rows per I slice (two per CTB row)
    int32_t i_seg_w;     // 16x16-unit columns per I slice (a CTB row in one or two segments)
    int32_t num_slices;
    int32_t aq;
    int32_t chroma_qp_offset;
    int32_t n_sse_parts;  // distortion partials written this frame (P: one per 4 CUs, I: one per CTU row)
    int32_t tu_split;     // inter split transform trees (EncoderConfig.tu_split: 1 8x8 nodes, 2 also 4x4 luma TUs)
    unsigned long long* sse_part;  // [3][kSsePartStride] per-workgroup distortion partials
    // temporal AQ classes (aq 3, h264_mb.h temporal_class): previous frame's source luma (read)
    // and this frame's copy (written by k_hevc_inter; IDR pictures copy it on the stream)
    const uint8_t* prev_src;
    uint8_t* save_src;
    // SAO (EncoderConfig::sao): the analysis kernels reconstruct into rec_*, deblocking filters
    // it in place, k_hevc_sao writes the final picture to sao_* (the reference of the next frame)
    int32_t sao;
    int32_t deblock_on;  // the in-loop filter runs on this picture (EncoderConfig::deblock 2: set by k_hevc_db_auto)
    uint8_t* sao_y;
    uint8_t* sao_uv;
    // quality-report mask in CTBs (x0, y0, x1, y1; x1 <= x0: none): k_hevc_sao adds a 4th
    // distortion channel, luma of the CTBs outside it (EncoderConfig::mask_*)
    int32_t mask_c[4];
    // k_hevc_sao's distortion totals (4 channels), accumulated with one atomic per workgroup and
    // channel; zeroed by k_hevc_layout earlier on the same stream
    unsigned long long* sse_tot;
    // wavefront parallel processing (EncoderConfig::hevc_wpp): one CABAC substream per CTU row; a
    // row's wave publishes its contexts after its second CTU (wpp_ctx[row][36 words], then
    // wpp_flag[row] = wpp_epoch with release semantics) and the next row's wave acquires them
    int32_t wpp;
    int32_t wpp_rows;    // CTU rows per P slice with WPP
    uint32_t wpp_epoch;  // nonzero, new every frame
    uint32_t* wpp_ctx;
    uint32_t* wpp_flag;
    int* wpp_err;  // mapped host word: nonzero if a substream gave up waiting for the row above
    // intra modes a CTB's first unit may use while its below-left is not reconstructed yet
    // (hevc_core.h bl_safe_modes: 16x16 luma and its DM 8x8 chroma)
    uint64_t bl_safe;
    uint64_t bl_safe_split;  // the same for a unit coded as four 8x8 TUs (hevc_core.h bl_safe_split)
    int32_t depth_inter;  // max_transform_hierarchy_depth_inter of the SPS
    int32_t deblock_auto;  // EncoderConfig::deblock 2: k_hevc_db_auto decides deblock_on (h264_deblock.h rule)
    int32_t chroma_keep;   // EncoderConfig::hevc_chroma_keep: changing content keeps its chroma residual
    int32_t depth_intra;   // max_transform_hierarchy_depth_intra of the SPS (1: intra units may split)
};

struct HevcOutHeader {
    uint32_t total_bytes;
    uint32_t num_slices;
    uint32_t overflow;
    uint32_t deblocked;  // the picture was deblocked (slice_deblocking_filter_disabled_flag 0)
    uint64_t sse[3];
    uint64_t sse_masked;  // luma outside the mask CTBs (SAO path; 0 otherwise)
    uint64_t t_start;     // device clock: k_hevc_publish (eager frames; 0 otherwise)
    uint64_t t_end;       // device clock: the last k_hevc_pack workgroup
};
static_assert(sizeof(HevcOutHeader) % 16 == 0, "payload must stay 16-byte aligned");
constexpr int kMaxSlices = 1024;
// k_hevc_sao distortion totals: kSseSlots slots of one 64-byte line each (workgroup w adds into
// slot w % kSseSlots), summed by k_hevc_pack
constexpr int kSseSlots = 64, kSseSlotWords = 8;
constexpr size_t kScanTilePad = 4096;  // per-CU scan arrays padded to this (hevc_kernels.hip kScanTile)
constexpr int kMaxSliceRows = 4;  // 16x16-unit rows per slice the intra wavefront kernel supports (2 CTB rows)
constexpr int kWppCtxWords = (C_NUM + 3) / 4;  // context states, four per dword
constexpr uint32_t kSubSliceStart = 0x80000000u;  // substream record: this substream begins a slice
// host buffer: header | substream payload offset[kMaxSlices] | length[] | first CTU[] | payloads
// (a substream is a slice without WPP, a CTU row of a slice with it)
constexpr size_t kOutPayloadOffset = sizeof(HevcOutHeader) + 3 * kMaxSlices * sizeof(uint32_t);

struct HevcDeviceBuffers {
    HevcFrameState* fs;
    h264::DeviceBuffers me;  // H.264 ME state (frame state + MbInfo with the motion vectors)
    CuInfo* cu;
    int16_t* coef;
    uint8_t* slice_data;     // [max_slices * slice_cap]
    uint32_t* slice_len;     // [max_slices]
    uint32_t slice_cap;
    int* slice_first;        // [max_slices] first CTB of every slice (k_hevc_layout)
    int* slice_of_cu;        // [nctb] slice of every CTB
    uint32_t* nslices;       // slice count of the frame
    uint8_t* qpy;            // [ncu] QpY per unit (deblocking)
    uint8_t* qp_pred;        // [ncu] QP predictor per unit (entropy coder)
    uint8_t* imode;          // [ncu] intra mode per unit (k_hevc_intra_modes, I pictures)
    uint32_t* cost;          // [nctb] CABAC cost estimate per CTB (slice layout)
    uint8_t* qpc;            // [ncu] QP of units that code a residual, else 255
    uint32_t* sao;           // [nctb][4] SAO parameters per CTB (hevc_core.h sao_pack; luma, Cb, Cr, 0)
    unsigned long long* slice_clk;  // [max_slices][2] k_hevc_arith start / end (wall_clock64, 100 MHz)
    uint16_t* tok;                  // [4 nctb][kMaxCuTokens] bin tokens per coding position (k_hevc_bins)
    uint32_t* ntok;                 // [4 nctb] token count per coding position (0 outside the picture)
    uint32_t* tok_off;              // [4 nctb + 1] exclusive prefix of ntok
    uint16_t* tok_dense;            // [4 nctb * kMaxCuTokens + 512] tokens in decoding order
    uint32_t* wpp_ctx;              // [ctb rows][kWppCtxWords] context snapshots (WPP)
    uint32_t* wpp_flag;             // [ctb rows] snapshot-ready epochs
    int* wpp_err;                   // mapped host word
    size_t out_bytes;
    unsigned long long* sse_part;
    unsigned long long* sse_tot;  // [kSseSlots][kSseSlotWords] k_hevc_sao distortion totals (4 used per slot)
    uint32_t* pack_done;          // [1] k_hevc_pack workgroups finished (the last stamps t_end, re-arms it)
    uint32_t* db_state;           // [4] adaptive filter: the last P decision, counters, ticket (shared by the slots)
};
// Eager frames: one kernel stores both frame states (kernel arguments) to the device and stamps
// the frame's start clock -- instead of two host-to-device copies (two blit kernels on the
// analysis stream) and a timing event.
void launch_hevc_publish(const HevcDeviceBuffers& b, const HevcFrameState& fs, const h264::FrameState* me_fs,
                         uint64_t* t_start, hipStream_t s);

// IDR + temporal AQ: the source luma into fs->save_src (pointer read on the device)
void launch_hevc_save_src(const Geometry& g, const HevcDeviceBuffers& b, const uint8_t* src_y, hipStream_t s);
void launch_hevc_inter(const Geometry& g, const HevcDeviceBuffers& b, const uint8_t* src_y, const uint8_t* src_uv,
                       hipStream_t s);
void launch_hevc_intra(const Geometry& g, const HevcDeviceBuffers& b, int slice_rows, int num_slices,
                       const uint8_t* src_y, const uint8_t* src_uv, hipStream_t s);
// Slice layout, per-slice decisions and (with deblock) the in-loop filter + final distortion:
// runs on the analysis stream because the deblocked picture is the next frame's reference.
// deblock_auto: k_hevc_db_auto decides the picture's filter first (EncoderConfig::deblock 2)
void launch_hevc_layout(const Geometry& g, const HevcDeviceBuffers& b, bool idr, int max_slices, int slice_cost, bool deblock,
                        bool sao, const uint8_t* src_y, const uint8_t* src_uv, hipStream_t s, bool deblock_auto = false);
void launch_hevc_entropy(const Geometry& g, const HevcDeviceBuffers& b, int max_slices, uint8_t* host_out,
                         hipStream_t s);

class GpuHevcEncoder final : public VideoEncoder {
   public:
    const char* codec() const override { return "hevc"; }
    h264::EncoderCommon& rc() override { return common_.rc(); }
    static constexpr int kMaxInFlight = 3;
    GpuHevcEncoder(const EncoderConfig& cfg, hipStream_t stream);
    ~GpuHevcEncoder();
    GpuHevcEncoder(const GpuHevcEncoder&) = delete;
    GpuHevcEncoder& operator=(const GpuHevcEncoder&) = delete;

    const Geometry& geometry() const override { return geom_; }
    int pitch() const override { return geom_.pitch; }
    int depth() const override { return depth_; }
    void submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr = false) override;
    const std::vector<uint8_t>& collect() override;
    const FrameStats& last_stats() const override { return stats_; }
    HevcCommon& common() { return common_; }
    const uint8_t* recon_y() const override { return rec_y_[cur_]; }
    const uint8_t* recon_uv() const override { return rec_uv_[cur_]; }
    hipEvent_t done_event() const override { return last_done_; }
    hipEvent_t pending_done_event() const override { return inflight_.empty() ? last_done_ : slots_[inflight_.front()].done; }
    // Per-slice CABAC timing of the last collected picture (diagnostics, synchronous copy):
    // (first CTU, CTUs, payload bytes, wave ticks at 100 MHz) per slice.
    // per substream of the last picture: first CTU, CTUs, bytes, wave ticks (100 MHz), start tick
    // relative to the earliest wave, tokens coded
    std::vector<std::array<uint64_t, 6>> slice_timing() const;
    // diagnostics: per-CU (type, cbf, sum of last+1, coded sub-blocks, est_bytes, tokens) of the last
    // collected picture (the CU cost model's calibration data, tools/hevc_session_timing.py)
    std::vector<std::array<uint32_t, 6>> cu_token_table() const;
   private:
    int mask_c_[4] = {0, 0, 0, 0};
    int64_t masked_pixels_ = 0;
   public:
    // split form (same as GpuH264Encoder) for the session's graph path
    bool prepare(bool force_idr) override;
    void enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) override;
    void record_start() override;
    void record_done() override;
    bool supports_split() const override { return true; }
    // masked luma distortion computed by k_hevc_sao (a mask is set and SAO is on)
    bool masked_sse_in_encoder() const override { return cfg_.sao != 0 && mask_c_[2] > mask_c_[0]; }
    int prep_slot() const override { return prep_slot_; }
    // one entropy stream per frame slot: the CABAC of consecutive frames is independent (only the
    // analysis chain carries the reference), so with 2-3 frames in flight their serial arithmetic
    // coders run side by side instead of queueing behind each other
    hipStream_t entropy_stream() const override { return stream_e_[prep_slot_]; }
    // frame GPU time from device clock stamps (the session's render stamp -> k_hevc_pack's end stamp)
    bool device_clock() const override { return true; }
    uint64_t last_t_end() const override { return last_t_end_; }
    void enqueue_analysis(bool idr, const uint8_t* src_y, const uint8_t* src_uv) override;
    void enqueue_entropy() override;
    void link_entropy() override;

   private:
    struct FrameSlot {
        HevcDeviceBuffers buf{};
        HevcFrameState* fs_host = nullptr;     // pinned
        h264::FrameState* me_fs_host = nullptr;  // pinned
        uint8_t* host_out = nullptr;           // pinned, mapped
        hipEvent_t start = nullptr, analysis_done = nullptr, done = nullptr;
        bool idr = false;
        int qp = 0;
        int poc = 0;
    };
    void alloc_slot(FrameSlot& sl);
    void free_slot(FrameSlot& sl);
    void fill_state(FrameSlot& sl, bool idr, int qp, int ref, int cur, bool probe = false);
    int probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp);

    EncoderConfig cfg_;
    HevcCommon common_;
    hipStream_t stream_;
    hipStream_t stream_e_[kMaxInFlight] = {};  // per slot (depth > 1; the first n_es_ own their stream)
    bool eager_ = false;        // submit(): states published by a kernel, device clock timing
    uint64_t last_t_end_ = 0;   // device clock at the end of the last collected frame
    double clock_khz_ = 100000;
    void enqueue_analysis_impl(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish);
    int n_es_ = 0;
    hipStream_t es(int slot) const { return stream_e_[slot] ? stream_e_[slot] : stream_; }
    int depth_ = 1;
    Geometry geom_;
    FrameSlot slots_[kMaxInFlight];
    int next_slot_ = 0, prep_slot_ = 0, last_slot_ = -1;
    std::vector<uint32_t> last_first_, last_len_;  // substream layout of the last collected picture
    uint32_t wpp_epoch_ = 0;
    std::deque<int> inflight_;
    hipEvent_t last_done_ = nullptr;
    uint8_t* hp_[4] = {nullptr, nullptr, nullptr, nullptr};
    int hp_pitch_ = 0;
    uint8_t* rec_y_[2] = {nullptr, nullptr};
    uint8_t* rec_uv_[2] = {nullptr, nullptr};
    uint8_t* src_keep_[2] = {nullptr, nullptr};  // source luma of the last two frames (temporal AQ classes)
    uint64_t bl_safe_ = 0;       // hevc_core.h bl_safe_modes (16x16 luma & DM chroma)
    uint64_t bl_safe_split_ = 0; // hevc_core.h bl_safe_split (8x8 luma & DM 4x4 chroma)
    uint8_t* pre_y_ = nullptr;   // SAO: reconstruction before SAO (deblocked in place)
    uint8_t* pre_uv_ = nullptr;
    uint32_t* db_state_ = nullptr;  // adaptive filter state (HevcDeviceBuffers::db_state)
    int cur_ = 0;
    bool have_ref_ = false;
    std::vector<uint8_t> au_;
    FrameStats stats_;
};

}  // namespace hevc
}  // namespace mx
