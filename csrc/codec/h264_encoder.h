// Host-side H.264 encoder API: GpuH264Encoder (HIP kernels, the production path) and
// CpuH264Encoder (same bitstream subset, serial C++ over the same core functions; used
// for the no-GPU "plumbing" configuration of BASELINE.json and as a bit-exact oracle
// for the GPU kernels in tests).
//
// Reference parity: WEBRTC_ENCODER selects nvh264enc (NVENC) or x264enc (CPU) in the
// reference (Dockerfile:210, README.md:21); here "mxh264enc" (GPU) / "cpuh264enc" (CPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "h264_core.h"
#include "h264_deblock.h"
#include "h264_gpu.h"
#include "video_encoder.h"

namespace mx {
namespace h264 {

struct EncoderConfig {
    int width = 1920;
    int height = 1080;
    int fps = 60;
    int bitrate_kbps = 8000;  // 0 = constant QP
    int qp = 28;              // initial / constant QP
    int qp_min = 18;
    int qp_max = 46;
    int keyint = 0;           // IDR period in frames, 0 = only on demand (infinite GOP)
    int search_range = 16;    // integer-pel full search radius (<= 32)
    int intra4x4 = 1;         // Intra4x4 allowed for intra MBs (0: Intra16x16 only -- cheaper IDR wavefront)
    int me_coarse = 0;        // 1: ME over the even-offset grid + the 8 integer neighbours of its best (4x
                              // fewer SADs: +5.7 % fps, -0.4 dB masked Y-PSNR at 8 Mbps, profiles/r02_me);
                              // 0: exhaustive +-range search
    int subpel = 1;           // quarter-pel refinement
    int chroma_qp_offset = 0;
    int aq = -1;              // adaptive quantisation of P macroblocks (mb_qp_delta): 1 coarser QP for
                              // noise-like residuals, 2 adds their rate-distortion residual drop, 3 temporal
                              // classes of the source -- persistent content 6 QP finer, changing content 6
                              // coarser, its chroma dropped and its luma residual kept only when it pays for
                              // its bits (h264_mb.h temporal_class); 4 (default), 5, 6: as 3 with static
                              // content (identical source, zero vector) 9 / 12 / 15 QP finer -- 4K desktop
                              // +0.6 dB (H.264) / +1.4 dB (HEVC) masked Y-PSNR at equal rate, motion content
                              // unchanged (profiles/r04_hevc/NOTES.md).  HEVC has 0, 1 and 3+, and treats 2
                              // as 1.  -1: the codec's default -- H.264 / VP8 4, HEVC 6 (4K 18 Mbps desktop
                              // +1.6 dB over aq 4, motion +0.1 dB, profiles/r05_hevc/NOTES.md)
    // in-loop deblocking filter: 1 on, 0 off, 2 adaptive (per picture from the coherent-motion
    // classes of the picture kDbLag back, h264_deblock.h db_auto_decide), -1 the codec's default --
    // HEVC adaptive (8.7.2 is fully parallel), H.264 adaptive (8.7 is a picture-wide wavefront,
    // k_deblock: on when at least a tenth of the picture moves coherently, where it gains 1.3 dB,
    // off on a mostly static desktop, where it gains 0.2 dB for -64 % single-session throughput;
    // paced density is 200 sessions either way, profiles/r06_defaults/NOTES.md), VP8 adaptive
    // too (section 15 is the same raster-order chain, k_vp8_lf: the desktop stays unfiltered at
    // the same rate, full-screen motion +0.8 dB for -15 % paced density / -74 % single-session
    // throughput, profiles/r06_vp8db/NOTES.md; vp8_encoder.h LfDecision)
    int deblock = -1;
    // P pictures: also search 16x8 / 8x16 partitionings (two vectors per macroblock) and take one
    // when its SAD + lambda * vector rate beats the 16x16 vector's
    int partitions = 1;
    // a copy with aq < 0 resolved to the codec's default (each encoder keeps one as cfg_)
    EncoderConfig with_aq_default(int def) const {
        EncoderConfig c = *this;
        if (c.aq < 0) c.aq = def;
        return c;
    }
    bool h264_deblock() const { return deblock != 0; }  // the filter kernels run (on, or adaptive)
    bool h264_deblock_auto() const { return deblock == 2 || deblock < 0; }
    int h264_deblock_mode() const { return deblock == 1 ? 1 : (deblock == 0 ? 0 : 2); }  // DbLagDecision mode
    bool hevc_deblock() const { return deblock != 0; }
    // HEVC's default is adaptive: deblocking costs the still desktop 0.3 dB (its text regions
    // 4.5 dB) and gains 0.2 dB on motion content at 4K 18 Mbps (profiles/r05_hevc/NOTES.md)
    bool hevc_deblock_auto() const { return deblock == 2 || deblock < 0; }
    int vp8_deblock_mode() const { return deblock == 1 || deblock == 2 ? deblock : (deblock < 0 ? 2 : 0); }
    int intra_in_p = 0;       // H.264: P-slice macroblocks may be coded intra (open-loop cost decision); off by
                              // default: it costs -35 % fps on the 1080p desktop (k_intra_analyze + k_intra_p on
                              // the analysis queue, profiles/r04_toolset/NOTES.md)
    int vp8_intra = 1;        // VP8 inter frames: intra macroblocks (two parallel passes, vp8_core.h
                              // vp8_intra_candidate)
    int vp8_bpred = 1;        // VP8 key frames: macroblocks may take B_PRED (16 4x4 sub-block modes, vp8_core.h
                              // bpred_luma) when its SAD + lambda * mode bits beat the 16x16 mode's
    int tu_split = 2;         // HEVC: inter transform trees may split into 8x8 luma / 4x4 chroma TUs (1), and each
                              // 8x8 luma node again into four 4x4 TUs (2), per node by SSE + lambda * bits
    // HEVC I pictures: a 16x16 intra unit may code its transform tree as four 8x8 luma / 4x4 chroma TUs,
    // each predicted from the reconstruction of the TUs before it (same mode; mode-dependent scans),
    // decided open-loop from the source (hevc_core.h intra_split_wins)
    int hevc_intra_split = 1;
    int hevc_slice_cost = 1536;  // HEVC without WPP: P-picture slice work target (hevc_core.h cu_cost units)
    // HEVC wavefront parallel processing (entropy_coding_sync_enabled_flag): P pictures in slices of
    // hevc_wpp_rows CTU rows, every CTU row its own CABAC substream (one GPU wave each) that starts
    // from the contexts the row above had after its second CTU.  Off by default: a CTU row is a
    // serial coder chain, and the rows through the desktop's detailed regions carry the most bins,
    // so at 4K / 25 Mbps WPP gave +0.27 dB masked for half the frame rate (817 vs 1,619 fps, with
    // 2- to 16-row slices all within 2 %: profiles/r04_hevc); cost-balanced slices split those
    // regions instead.  0: cost-balanced slices, one substream per slice
    int hevc_wpp = 0;
    // HEVC with WPP: CTU rows per P slice (0 = the whole picture).  A substream row is a serial
    // chain and a slice's rows start two CTUs apart, so a slice of R rows takes ~2R + row-length
    // CTU times: short slices keep the wavefront's fill out of the frame time (at 4K one slice
    // took ~3 ms of CABAC waves, 8-row slices ~1.4 ms; profiles/r04_hevc)
    int hevc_wpp_rows = 8;
    int sao = 1;              // HEVC: sample adaptive offset (8.7.3), band / edge offsets decided per CTB
    // HEVC, aq >= 3: changing content (video, animation) keeps its residual, chroma included, coded
    // at its class QP, instead of the chroma drop and the luma rate-distortion drop
    int hevc_chroma_keep = 0;
    // quality report: luma distortion outside the macroblocks touching this pixel rectangle
    // (FrameStats::sse_masked; mask_x1 <= mask_x0 = no mask)
    int mask_x0 = 0, mask_y0 = 0, mask_x1 = 0, mask_y1 = 0;
    int pipeline_depth = 1;   // GPU frames in flight: 2 overlaps frame n's entropy coding with
                              // frame n+1's analysis on a second HIP stream (rate control lags a frame);
                              // 3 also keeps the next frame's launches queued while the host collects
                              // frame n (the host turnaround then overlaps GPU work; H.264 / HEVC)
};

struct FrameStats {
    int64_t frame_index = 0;
    int idr = 0;
    int qp = 0;
    int bytes = 0;
    int skipped_mbs = 0;
    double encode_ms = 0;
    uint64_t sse[3] = {0, 0, 0};  // source vs reconstruction (Y, U, V), display area
    uint64_t sse_masked = 0;      // Y outside the mask macroblocks (EncoderConfig::mask_*)
    int64_t masked_pixels = 0;    // display luma samples outside them (the PSNR denominator)
    int deblocked = 0;            // the in-loop filter ran on this picture (H.264 idc 0, HEVC, VP8 level > 0)
    int db_coherent = 0, db_changed = 0, db_moving = 0;  // adaptive filter: the picture's class counts (db_auto_count)
};

// Annex-B / rate-control logic shared by both encoders.
//
// Rate control (CBR, bitrate_kbps > 0) is a per-frame bit-budget controller with a virtual
// buffer (VBV) model, replacing the reference's NVENC low-latency CBR (`nvh264enc`,
// reference Dockerfile:210):
//  * rate model per picture type t in {I, P}: bits = X_t / qstep(QP)^a, qstep = 0.625*2^(QP/6);
//    X_t is re-estimated from every finished frame, the P slope `a` from consecutive P frames
//    at different QPs (tuned offline on measured rate-QP curves: tools/rc_trace.py);
//  * the very first IDR is sized by a synchronous probe encode (wants_probe()/add_probe()),
//    so the stream starts on budget instead of converging for a second;
//  * every IDR gets its own budget (idr_budget x the per-frame budget) and IS charged to the
//    buffer; the excess is drained over the next kDrainFrames P frames (bounded recovery);
//  * frames in flight (pipelined encode) are charged at their budget until they finish.
class EncoderCommon {
   public:
    explicit EncoderCommon(const EncoderConfig& c);
    const EncoderConfig& config() const { return cfg_; }
    int mb_w() const { return mb_w_; }
    int mb_h() const { return mb_h_; }
    // Decide frame type/params for the next frame.
    void begin_frame(bool force_idr);
    bool cur_idr() const { return cur_idr_; }
    int cur_qp() const { return cur_qp_; }
    int cur_frame_num() const { return frame_num_; }
    int cur_idr_pic_id() const { return idr_pic_id_; }
    int log2_max_frame_num() const { return 8; }
    int pic_init_qp() const { return 26; }
    // Append SPS/PPS NAL units (Annex-B) to out.
    void write_parameter_sets(std::vector<uint8_t>& out) const;
    // Append one slice NAL (start code + header byte + emulation-prevented payload).
    void write_slice_nal(std::vector<uint8_t>& out, const uint8_t* rbsp, size_t n, bool idr) const;
    // Update rate control after a frame of `bytes` bytes (frames end in begin order).
    void end_frame(int bytes, bool idr);
    void request_idr() { idr_requested_ = true; }
    void set_bitrate(int kbps) { cfg_.bitrate_kbps = kbps; }
    int64_t frames() const { return frame_index_; }

    // ---- rate-control internals (exposed for the encoders and tests)
    static double qstep(double qp) { return 0.625 * std::exp2(qp / 6.0); }
    double frame_budget_bits() const;  // bitrate / fps
    // True while the first IDR of a CBR stream still wants a probe encode.
    bool wants_probe() const { return cfg_.bitrate_kbps > 0 && begun_ == 0 && probes_ < kMaxProbes && !probe_done_; }
    int probe_qp() const;                 // QP to probe next
    void add_probe(int qp, int bytes);    // result of a probe encode of the first picture
    double vbv_excess_bits() const { return vbv_; }
    static constexpr int kDrainFrames = 4;
    static constexpr double kPPrior = 0.3;  // first P picture after an IDR: bits ~ kPPrior x the IDR's at equal QP
    static constexpr double kIdrBudget = 5.0;  // IDR budget in frames (tools/region_report.py sweep)
    static constexpr int kMaxProbes = 2;
    static constexpr int kMaxStep = 4;  // max P-picture QP rise per frame (damps the pipelined loop)
    static constexpr int kMaxDown = 3;  // max P-picture QP fall per frame (bounds refinement spikes)

   private:
    int qp_for(double x, double bits, double alpha) const;
    EncoderConfig cfg_;
    int mb_w_, mb_h_;
    bool cur_idr_ = true;
    bool idr_requested_ = true;
    int cur_qp_;
    int frame_num_ = 0;
    int idr_pic_id_ = -1;
    int64_t frame_index_ = 0;  // frames ended
    int64_t begun_ = 0;        // frames begun
    int64_t since_idr_ = 0;    // frames begun since (and including) the last IDR
    // rate model / buffer
    double x_i_ = 0, x_p_ = 0;  // complexity (bits * qstep^alpha) of I / P pictures; 0 = unknown
    double alpha_p_ = 1.0;      // P rate-QP slope, re-estimated from consecutive P pictures
    double prev_p_bits_ = 0;
    int prev_p_qp_ = -1;
    int last_i_qp_ = -1, last_p_qp_ = -1;  // last_p_qp_: QP of the last begun picture (IDR included)
    bool last_was_idr_ = false;
    double vbv_ = 0;  // bits sent above the CBR line so far (>= -1 frame budget)
    struct Pending {
        double budget;
        int qp;
        bool idr;
        int64_t since_idr;  // frames since the IDR (1 = the IDR itself)
    };
    std::deque<Pending> pending_;  // begun, not yet ended (pipelined frames)
    int probes_ = 0;
    bool probe_done_ = false;
    int probe_q_[kMaxProbes] = {0, 0};
};

void emulation_prevent(std::vector<uint8_t>& out, const uint8_t* rbsp, size_t n);
// Test hook: run k_hpel on a host reference picture; returns the padded F/H/V/J planes
// (origin at (kHpelPad, kHpelPad), pitch in *hp_pitch).
std::vector<std::vector<uint8_t>> hpel_planes_for_test(const uint8_t* ref, int coded_w, int coded_h, int pitch,
                                                       int* hp_pitch);

class GpuH264Encoder final : public VideoEncoder {
   public:
    const char* codec() const override { return "h264"; }
    EncoderCommon& rc() override { return common_; }
    static constexpr int kMaxInFlight = 4;
    GpuH264Encoder(const EncoderConfig& cfg, hipStream_t stream);
    ~GpuH264Encoder();
    GpuH264Encoder(const GpuH264Encoder&) = delete;
    GpuH264Encoder& operator=(const GpuH264Encoder&) = delete;

    const Geometry& geometry() const override { return geom_; }
    int pitch() const override { return geom_.pitch; }
    hipStream_t stream() const { return stream_; }
    int depth() const override { return depth_; }
    int in_flight() const { return (int)inflight_.size(); }

    // Enqueue the encode of an NV12 frame already in device memory (pitch = pitch()).
    // Equivalent to prepare() + record_start() + enqueue_body() + record_done().  With
    // pipeline_depth 2 a second frame may be submitted before the first is collected:
    // analysis (hpel/ME/inter or intra) runs on `stream`, entropy coding (CAVLC/scan/pack) on
    // an internal stream, so frame n's entropy coding overlaps frame n+1's analysis.
    void submit(const uint8_t* src_y, const uint8_t* src_uv, bool force_idr = false) override;
    // Wait for the oldest submitted frame and return its Annex-B access unit.
    const std::vector<uint8_t>& collect() override;
    const FrameStats& last_stats() const override { return stats_; }
    EncoderCommon& common() { return common_; }
    // Reconstructed frame of the last prepared picture (device pointers).
    const uint8_t* recon_y() const override { return rec_y_[cur_]; }
    const uint8_t* recon_uv() const override { return rec_uv_[cur_]; }
    // Split form for hipGraph replay (depth 1): host-side frame decisions (rate control,
    // reference swap) into the pinned frame state; returns whether this is an IDR frame.
    bool prepare(bool force_idr) override;
    // Frame-state upload + kernels (stream-capturable; identical every frame of a type).
    void enqueue_body(bool idr, const uint8_t* src_y, const uint8_t* src_uv) override;
    void record_start() override;
    void record_done() override;
    // depth-2 graph form (VideoEncoder): deblocking needs an extra event inside the entropy
    // chain, so the split form is offered only with the filter off (Session sets it off for graphs)
    bool supports_split() const override { return !cfg_.h264_deblock(); }
    bool masked_sse_in_encoder() const override { return true; }
    int prep_slot() const override { return prep_slot_; }
    hipStream_t entropy_stream() const override { return stream_e_; }
    void enqueue_analysis(bool idr, const uint8_t* src_y, const uint8_t* src_uv) override;
    void enqueue_entropy() override;
    void link_entropy() override;
    void set_hpel_side_stream(bool on) override;
    void quiesce() override { drain_launcher(); }
    // P pictures: the wait goes after k_hpel (which reads only the reference), so the
    // interpolation of the new reference runs without waiting for the capture hand-off
    bool set_input_event(hipEvent_t ev) override {
        in_ev_ = ev;
        return true;
    }
    // Completion event of the last collected frame.
    hipEvent_t done_event() const override { return last_done_; }
    bool device_clock() const override { return true; }
    uint64_t last_t_end() const override { return last_t_end_; }
    hipEvent_t pending_done_event() const override {
        if (inflight_.empty()) return last_done_;
        wait_launched(inflight_.front());  // the launcher thread has recorded it
        return slots_[inflight_.front()].done;
    }
    // publish: the first kernel takes the frame state by value and stores it (eager launches);
    // otherwise the kernels read the device copy uploaded by enqueue_body's memcpy node.
    void enqueue_kernels(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish);
    void enqueue_analysis_kernels(bool idr, const uint8_t* src_y, const uint8_t* src_uv, bool publish);

   private:
    struct FrameSlot {  // per-frame-in-flight state
        DeviceBuffers buf{};
        FrameState* fs_host = nullptr;  // pinned
        uint8_t* host_out = nullptr;    // pinned, mapped: OutHeader | slice tables | payload
        hipEvent_t start = nullptr, analysis_done = nullptr, deblock_done = nullptr, done = nullptr;
        hipEvent_t hpel_done = nullptr;
        bool idr = false;
        bool deblock = false;  // the picture's in-loop filter (decided when it is prepared)
        bool me_unf = false;   // the reference was deblocked: the search uses its unfiltered planes (hpu_)
        int qp = 0;
        uint64_t fidx = 0;     // picture number (seq_ when prepared)
        hipEvent_t me_done = nullptr;  // the side-stream motion search of this picture
    };
    void alloc_slot(FrameSlot& sl);
    void free_slot(FrameSlot& sl);
    void fill_state(FrameSlot& sl, bool idr, int qp, int ref, int cur);
    void unfiltered_planes(FrameSlot& sl);
    int probe_bytes(const uint8_t* src_y, const uint8_t* src_uv, int qp);
    // Entropy launcher (depth > 1, eager launches): a thread issues each frame's entropy chain --
    // the wait for its analysis, the CAVLC / scan / pack launches and its completion event, all
    // on the entropy stream -- while the calling thread returns to the next frame's capture and
    // analysis launches (the host launch sequence bounds the single-session rate,
    // profiles/r04_capture).  MXDESK_ENTROPY_THREAD=0 keeps every launch on the calling thread.
    struct EntropyJob {
        int slot;
        hipEvent_t sse_ready;
    };
    void launcher_loop();
    void wait_launched(int slot) const;  // the job that records slots_[slot].done was issued
    void drain_launcher() const;         // every queued job issued
    std::thread launcher_;
    mutable std::mutex lmu_;
    mutable std::condition_variable lcv_;
    std::deque<EntropyJob> ljobs_;
    uint64_t l_pushed_ = 0, l_done_ = 0;
    uint64_t slot_job_[kMaxInFlight] = {};  // job number that records the slot's done event (0: none)
    bool lstop_ = false;
    std::exception_ptr lerr_;
    bool sync_launch_ = false;  // probe: everything on the calling thread
    bool async_frame_ = false;  // the frame being submitted went to the launcher
    int device_ = 0;

    EncoderConfig cfg_;
    EncoderCommon common_;
    hipStream_t stream_;
    hipStream_t stream_e_ = nullptr;  // entropy stream (depth 2)
    // depth > 1, eager launches: k_hpel of a P picture runs on its own stream as soon as the
    // reference is final (ref_ready_, recorded after the previous picture's last reconstruction
    // kernel), beside the capture and colour conversion of the new picture, which it does not
    // depend on; k_me_full waits for it (profiles/r04_h264)
    hipStream_t stream_a_ = nullptr;
    bool hpel_side_ = true;  // set_hpel_side_stream
    hipEvent_t in_ev_ = nullptr;  // set_input_event, consumed by the next analysis launch
    hipEvent_t ref_ready_ = nullptr;
    uint64_t seq_ = 0, ref_seq_ = ~0ull;  // pictures prepared; the one whose reconstruction ref_ready_ marks
    int depth_ = 1;
    Geometry geom_;
    FrameSlot slots_[kMaxInFlight];
    int next_slot_ = 0, prep_slot_ = 0;
    std::deque<int> inflight_;
    hipEvent_t last_done_ = nullptr;
    uint64_t last_t_end_ = 0;   // device clock at the end of the last collected frame
    double clock_khz_ = 100000;  // device wall-clock rate
    uint8_t* hp_[4] = {nullptr, nullptr, nullptr, nullptr};  // padded F/H/V/J reference planes
    // With the in-loop filter on, the motion search of picture n+1 reads the F/H/V/J planes of
    // picture n's reconstruction before the filter (hpu_, k_hpel right after the reconstruction)
    // and runs on stream_m_ beside picture n's k_deblock; the analysis stream waits for it only
    // before k_inter_encode (whose prediction uses the filtered planes hp_)
    uint8_t* hpu_[4] = {nullptr, nullptr, nullptr, nullptr};
    hipStream_t stream_m_ = nullptr;
    hipEvent_t ev_hpu_ = nullptr;  // hpu_ of the last deblocked picture written
    bool last_deblock_ = false;    // the last prepared picture is deblocked
    int hp_pitch_ = 0;
    uint8_t* rec_y_[2] = {nullptr, nullptr};
    uint8_t* rec_uv_[2] = {nullptr, nullptr};
    uint8_t* src_keep_[2] = {nullptr, nullptr};  // source luma of the last two frames (temporal AQ classes)
    int cur_ = 0;  // index of the frame being reconstructed
    bool have_ref_ = false;
    uint32_t db_epoch_ = 0;
    // adaptive filter: picture n's decision from the classes of picture n - kDbLag (OutHeader::db_*,
    // recorded when it is collected); a picture's filter is fixed when it is prepared (FrameSlot::deblock)
    DbLagDecision db_lag_;
    int mask_mb_[4] = {0, 0, 0, 0};  // quality-report mask in macroblocks (x0, y0, x1, y1)
    int64_t masked_pixels_ = 0;
    std::vector<uint8_t> au_;
    FrameStats stats_;
};

class CpuH264Encoder {
   public:
    explicit CpuH264Encoder(const EncoderConfig& cfg);
    // Encode an NV12 frame (host memory, luma pitch == uv pitch == `pitch`, at least the
    // coded size mb_w*16 x mb_h*16 readable; use pad_nv12() for display-sized frames).
    const std::vector<uint8_t>& encode(const uint8_t* y, const uint8_t* uv, int pitch, bool force_idr = false);
    const FrameStats& last_stats() const { return stats_; }
    EncoderCommon& common() { return common_; }
    const std::vector<uint8_t>& recon_y() const { return rec_y_[cur_]; }
    const std::vector<uint8_t>& recon_uv() const { return rec_uv_[cur_]; }
    int coded_pitch() const { return cw_; }
    // analysis hooks: per-MB coded bits of the last frame (0 = skipped) and the MB records
    const std::vector<uint32_t>& mb_bits() const { return mb_bits_; }
    const std::vector<MbInfo>& mb_info() const { return mb_; }

   private:
    void encode_intra(const uint8_t* y, const uint8_t* uv, int pitch);
    void encode_inter(const uint8_t* y, const uint8_t* uv, int pitch);
    void entropy(std::vector<uint8_t>& payload, std::vector<uint32_t>& slice_off, std::vector<uint32_t>& slice_len);
    int frame_qp_() const { return qp_override_ >= 0 ? qp_override_ : common_.cur_qp(); }
    // the picture's in-loop filter (EncoderConfig::deblock; adaptive: DbLagDecision on the classes of
    // picture n - kDbLag, as the GPU encoder's host side) / the record of this picture's classes
    void decide_deblock();
    void update_deblock_decision();
    bool deblock_now_ = false;
    bool ref_deblocked_ = false;       // the reference picture was deblocked: search its unfiltered copy
    std::vector<uint8_t> rec_unf_y_;   // the last picture's luma reconstruction before the filter
    DbLagDecision db_lag_;
    uint64_t enc_seq_ = 0;  // pictures encoded (the GPU encoder's seq_)
    DbAutoCounts db_counts_;
    int qp_override_ = -1;  // rate-control probe of the first picture

    EncoderConfig cfg_;
    EncoderCommon common_;
    int cw_, ch_;
    std::vector<uint8_t> rec_y_[2], rec_uv_[2];
    int cur_ = 0;
    bool have_ref_ = false;
    std::vector<MbInfo> mb_;
    std::vector<int16_t> coef_;
    std::vector<uint32_t> mb_bits_;
    std::vector<uint8_t> prev_src_;  // previous source luma (coded size), temporal AQ classes
    std::vector<uint8_t> au_;
    FrameStats stats_;
};

// CPU motion search of one 16x16 block (same rules as the GPU k_me_full); shared by the
// CPU H.264 and HEVC encoders.
void me_search_cpu(const uint8_t* sy, int pitch, const uint8_t* ref_y, int cw, int ch, int x0, int y0, int qp,
                   int search_range, int subpel, int* mvx, int* mvy, int coarse);
// The same search plus 16x8 / 8x16 partitionings (k_me_full with FrameState::partitions): writes
// m.mvx / mvy (best 16x16 vector), m.part and m.pmv.
void me_search_parts_cpu(const uint8_t* sy, int pitch, const uint8_t* ref_y, int cw, int ch, int x0, int y0, int qp,
                         int search_range, int subpel, int coarse, MbInfo& m);

// Pad a display-sized NV12 frame to the coded size by edge replication (what the CSC
// kernel does on the GPU side).  Returns pitch = coded width.
void pad_nv12(const uint8_t* y, const uint8_t* uv, int w, int h, int pitch, int coded_w, int coded_h,
              std::vector<uint8_t>& oy, std::vector<uint8_t>& ouv);

}  // namespace h264
}  // namespace mx
