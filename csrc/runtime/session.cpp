#include "session.h"

#include <functional>
#include <cstdio>
#include <cstdlib>

#include <exception>
#include <thread>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../common/hip_check.h"
#include "../common/trace.h"
#include "../codec/hevc_encoder.h"
#include "../codec/vp8_encoder.h"

namespace mx {

// ------------------------------------------------------------------ FramePool
FramePool::FramePool(int width, int height, int slots) : w_(width), h_(height) {
    if (slots < 1) throw std::invalid_argument("FramePool needs >= 1 slot");
    pitch_ = ((width * 4) + 255) & ~255;
    buf_.resize(slots, nullptr);
    gen_.assign(slots, 0);
    for (auto& b : buf_) HIP_CHECK(hipMalloc(&b, (size_t)pitch_ * height));
}

FramePool::~FramePool() {
    for (auto b : buf_) hipFree(b);
}

int FramePool::acquire() {
    const int s = next_;
    next_ = (next_ + 1) % (int)buf_.size();
    gen_[s] = ++counter_;
    return s;
}

// ------------------------------------------------------------------ Lanczos tables
static double lanczos3(double x) {
    x = std::fabs(x);
    if (x < 1e-9) return 1.0;
    if (x >= 3.0) return 0.0;
    const double px = M_PI * x;
    return 3.0 * std::sin(px) * std::sin(px / 3.0) / (px * px);
}

void make_lanczos_table(int in_size, int out_size, std::vector<int>& start, std::vector<float>& weights, int& taps) {
    const double s = (double)in_size / out_size;
    const double f = std::max(1.0, s);
    const double support = 3.0 * f;
    taps = (int)std::ceil(2.0 * support) + 1;
    start.resize(out_size);
    weights.assign((size_t)out_size * taps, 0.f);
    for (int o = 0; o < out_size; ++o) {
        const double center = (o + 0.5) * s - 0.5;
        const int x0 = (int)std::floor(center - support) + 1;
        start[o] = x0;
        double sum = 0;
        std::vector<double> w(taps);
        for (int k = 0; k < taps; ++k) {
            w[k] = lanczos3((x0 + k - center) / f);
            sum += w[k];
        }
        for (int k = 0; k < taps; ++k) weights[(size_t)o * taps + k] = (float)(w[k] / sum);
    }
}

// ------------------------------------------------------------------ Session
int64_t Session::now_us() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

Session::Session(const SessionConfig& cfg) : cfg_(cfg) {
    if (cfg_.out_width <= 0) cfg_.out_width = cfg_.width;
    if (cfg_.out_height <= 0) cfg_.out_height = cfg_.height;
    cfg_.enc.width = cfg_.out_width;
    cfg_.enc.height = cfg_.out_height;
    cfg_.enc.fps = cfg_.fps;
    // the H.264 encoder reports the masked distortion itself (a 4th channel of its per-MB
    // partials, MB-aligned mask); other codecs use the separate k_sse_masked pass
    cfg_.enc.mask_x0 = cfg_.mask_x0;
    cfg_.enc.mask_y0 = cfg_.mask_y0;
    cfg_.enc.mask_x1 = cfg_.mask_x1;
    cfg_.enc.mask_y1 = cfg_.mask_y1;
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    pool_ = std::make_unique<FramePool>(cfg_.width, cfg_.height, cfg_.pool_slots);
    if ((cfg_.codec == "h264" || cfg_.codec == "avc") && cfg_.use_graph && cfg_.enc.deblock != 0 &&
        cfg_.enc.deblock != 1) {
        // the adaptive filter changes the picture's kernel sequence, a replayed graph cannot:
        // graph replay takes the filter off unless it is set on for every picture
        if (cfg_.enc.deblock > 1)
            throw std::invalid_argument("hipGraph replay needs a fixed H.264 filter (deblock 0 or 1), not adaptive");
        cfg_.enc.deblock = 0;
    }
    if (cfg_.codec == "h264" || cfg_.codec == "avc")
        enc_ = std::make_unique<h264::GpuH264Encoder>(cfg_.enc, stream_);
    else if (cfg_.codec == "hevc" || cfg_.codec == "h265")
        enc_ = std::make_unique<hevc::GpuHevcEncoder>(cfg_.enc, stream_);
    else if (cfg_.codec == "vp8")
        enc_ = std::make_unique<vp8::GpuVp8Encoder>(cfg_.enc, stream_);
    else
        throw std::invalid_argument("Session: unknown codec '" + cfg_.codec + "' (h264 | hevc | vp8)");
    const h264::Geometry& g = enc_->geometry();
    depth_ = enc_->depth();
    if (depth_ > kMaxDepth) throw std::invalid_argument("Session: encoder pipeline depth above kMaxDepth");
    for (int k = 0; k < depth_; ++k) {
        HIP_CHECK(hipMalloc(&nv12_y_[k], (size_t)g.pitch * g.coded_h));
        HIP_CHECK(hipMalloc(&nv12_uv_[k], (size_t)g.pitch * g.coded_h / 2));
    }
    const std::string codec = enc_->codec();
    const bool cap = cfg_.capture_stream > 0 || (cfg_.capture_stream < 0 && (codec == "h264" || codec == "hevc"));
    if (depth_ > 1 && cap && !cfg_.use_graph) {
        // MXDESK_CAPTURE_PRIORITY=low: the capture stream at the lowest priority, so its render /
        // conversion kernels yield compute units to the previous frame's analysis (4K H.264
        // 4,491 -> 4,613 fps).  Not the default: a stream of another priority takes a hardware
        // queue of its own for the whole process, and the other sessions' streams then share
        // fewer queues (paced density 200 -> 136 sessions, profiles/r04_capture)
        const char* cp = std::getenv("MXDESK_CAPTURE_PRIORITY");
        if (cp && std::string(cp) == "low") {
            int least = 0, greatest = 0;
            HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIP_CHECK(hipStreamCreateWithPriority(&cap_stream_, hipStreamNonBlocking, least));
        } else {
            HIP_CHECK(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking));
        }
        for (int k = 0; k < depth_; ++k)  // GPU-to-GPU only: device-scope release
            HIP_CHECK(hipEventCreateWithFlags(&ev_conv_[k], hipEventDisableTiming | hipEventReleaseToDevice));
        enc_->set_hpel_side_stream(false);
    }
    if (depth_ > 1 && cfg_.use_graph && !enc_->supports_split())
        throw std::invalid_argument("hipGraph replay with pipeline_depth 2 needs an encoder with the split form");
    if (depth_ >= cfg_.pool_slots) throw std::invalid_argument("pool_slots must exceed pipeline_depth");
    for (int k = 0; k < depth_; ++k)
        HIP_CHECK(hipHostMalloc(&staging_[k], (size_t)pool_->pitch() * cfg_.height, hipHostMallocDefault));
    scale_ = cfg_.out_width != cfg_.width || cfg_.out_height != cfg_.height;
    if (scale_) {
        std::vector<int> sx, sy;
        std::vector<float> wx, wy;
        int tx, ty;
        make_lanczos_table(cfg_.width, cfg_.out_width, sx, wx, tx);
        make_lanczos_table(cfg_.height, cfg_.out_height, sy, wy, ty);
        const size_t bytes = (sx.size() + sy.size()) * 4 + (wx.size() + wy.size()) * 4;
        HIP_CHECK(hipMalloc(&lt_mem_, bytes));
        char* p = static_cast<char*>(lt_mem_);
        lt_.out_w = cfg_.out_width;
        lt_.out_h = cfg_.out_height;
        lt_.taps_x = tx;
        lt_.taps_y = ty;
        lt_.x0 = reinterpret_cast<const int*>(p);
        HIP_CHECK(hipMemcpy(p, sx.data(), sx.size() * 4, hipMemcpyHostToDevice));
        p += sx.size() * 4;
        lt_.y0 = reinterpret_cast<const int*>(p);
        HIP_CHECK(hipMemcpy(p, sy.data(), sy.size() * 4, hipMemcpyHostToDevice));
        p += sy.size() * 4;
        lt_.wx = reinterpret_cast<const float*>(p);
        HIP_CHECK(hipMemcpy(p, wx.data(), wx.size() * 4, hipMemcpyHostToDevice));
        p += wx.size() * 4;
        lt_.wy = reinterpret_cast<const float*>(p);
        HIP_CHECK(hipMemcpy(p, wy.data(), wy.size() * 4, hipMemcpyHostToDevice));
        // matrix-core form of the scaler (falls back to the VALU kernel outside its range)
        const h264::Geometry& eg = enc_->geometry();
        pix::ScaleFragsHost fr;
        if (!cfg_.scale_valu && pix::build_scale_frags(cfg_.width, cfg_.height, cfg_.out_width, cfg_.out_height,
                                                       eg.coded_w, eg.coded_h, sx, wx, tx, sy, wy, ty, fr))
            pix::upload_scale_frags(fr, &lt_mf_mem_, lt_.mf);
    }
    for (int k = 0; k < kMaxDepth; ++k) HIP_CHECK(hipEventCreate(&ev_start_[k]));
    devclk_ = enc_->device_clock();
    clock_khz_ = device_clock_khz();
    HIP_CHECK(hipHostMalloc(&ts_, sizeof(uint64_t) * cfg_.pool_slots, hipHostMallocMapped));
    std::memset(ts_, 0, sizeof(uint64_t) * cfg_.pool_slots);
    mask_in_encoder_ = enc_->masked_sse_in_encoder();
    if (masked() && !mask_in_encoder_) {
        const h264::Geometry& eg = enc_->geometry();
        const int nb = pix::sse_masked_blocks(eg.width, eg.height);
        HIP_CHECK(hipMalloc(&mask_dev_, kMaxDepth * (size_t)nb * sizeof(unsigned long long)));
        HIP_CHECK(hipMalloc(&mask_counter_, kMaxDepth * sizeof(unsigned int)));
        HIP_CHECK(hipMemset(mask_counter_, 0, kMaxDepth * sizeof(unsigned int)));
        mask_stride_ = nb;
        HIP_CHECK(hipHostMalloc(&mask_host_, kMaxDepth * sizeof(unsigned long long), hipHostMallocMapped));
        for (int k = 0; k < kMaxDepth; ++k) HIP_CHECK(hipEventCreateWithFlags(&ev_mask_[k], hipEventDisableTiming));
    }
    // one parameter block per frame slot: with two frames in flight a captured memcpy node may
    // run after the host has already written the next frame's parameters
    HIP_CHECK(hipHostMalloc(&synth_host_, sizeof(pix::SynthParams) * cfg_.pool_slots, hipHostMallocDefault));
    // static layer of the synthetic desktop, rendered once (k_synth copies it outside the
    // animated elements)
    HIP_CHECK(hipMalloc(&synth_bg_, (size_t)pool_->pitch() * cfg_.height));
    pix::launch_synth_static(synth_bg_, synth_params(), stream_);
    HIP_CHECK(hipGetLastError());
    // k_synth reads the static layer from cap_stream_ (a non-blocking stream with no order
    // against stream_) or from the upload stream: the layer must be complete before the first
    // frame is rendered on any of them
    HIP_CHECK(hipStreamSynchronize(stream_));
    HIP_CHECK(hipMalloc(&synth_dev_, sizeof(pix::SynthParams) * cfg_.pool_slots));
    // [frame slot][encoder slot][IDR][analysis, entropy]
    graphs_.assign((size_t)cfg_.pool_slots * kMaxDepth * 2 * 2, nullptr);
    t0_us_ = now_us();
}

Session::~Session() {
    if (ht_n_ > 0 && std::getenv("MXDESK_HOST_TIMING"))
        std::fprintf(stderr, "[mxdesk] host us/frame over %lld frames: submit %.1f, wait %.1f, collect %.1f\n",
                     (long long)ht_n_, ht_submit_ / ht_n_, ht_wait_ / ht_n_, ht_post_ / ht_n_);
    // drain every stream that can still touch the pinned stamp block, the synth parameters or
    // the static layer (frames in flight on the capture / upload streams and in the encoder)
    // before anything is freed
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (cap_stream_) (void)hipStreamSynchronize(cap_stream_);
    if (upload_stream_) (void)hipStreamSynchronize(upload_stream_);
    enc_.reset();
    for (auto g : graphs_)
        if (g) hipGraphExecDestroy(g);
    hipHostFree(synth_host_);
    if (ts_) hipHostFree(ts_);
    if (synth_bg_) hipFree(synth_bg_);
    hipFree(synth_dev_);
    pool_.reset();
    if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
    for (int k = 0; k < kMaxDepth; ++k) {
        if (nv12_y_[k]) (void)hipFree(nv12_y_[k]);
        if (nv12_uv_[k]) (void)hipFree(nv12_uv_[k]);
        if (ev_conv_[k]) (void)hipEventDestroy(ev_conv_[k]);
    }
    for (int k = 0; k < kMaxDepth; ++k)
        if (staging_[k]) (void)hipHostFree(staging_[k]);
    if (lt_mem_) hipFree(lt_mem_);
    if (lt_mf_mem_) hipFree(lt_mf_mem_);
    for (const auto& r : host_regs_) (void)hipHostUnregister(const_cast<uint8_t*>(r.first));
    if (screen_) (void)hipFree(screen_);
    if (ev_upload_) (void)hipEventDestroy(ev_upload_);
    if (upload_stream_) {
        (void)hipStreamSynchronize(upload_stream_);
        (void)hipStreamDestroy(upload_stream_);
    }
    for (int k = 0; k < kMaxDepth; ++k) (void)hipEventDestroy(ev_start_[k]);
    if (mask_dev_) (void)hipFree(mask_dev_);
    if (mask_counter_) (void)hipFree(mask_counter_);
    if (mask_host_) (void)hipHostFree(mask_host_);
    for (int k = 0; k < kMaxDepth; ++k)
        if (ev_mask_[k]) (void)hipEventDestroy(ev_mask_[k]);
    hipStreamDestroy(stream_);
}

void Session::convert(int slot, hipStream_t st, uint64_t* ts) {
    const h264::Geometry& g = enc_->geometry();
    uint8_t* y = nv12_y_[cur_k_];
    uint8_t* uv = nv12_uv_[cur_k_];
    if (scale_) {
        pix::launch_scale_to_nv12(pool_->data(slot), pool_->pitch(), cfg_.width, cfg_.height, lt_, y, uv, g.pitch,
                                  g.coded_w, g.coded_h, st, ts);
    } else {
        pix::launch_bgrx_to_nv12(pool_->data(slot), pool_->pitch(), cfg_.width, cfg_.height, y, uv, g.pitch,
                                 g.coded_w, g.coded_h, st, ts);
    }
    HIP_CHECK(hipGetLastError());
}

void Session::convert_and_encode(int slot, bool force_idr, bool stamp) {
    TraceRange tr("mxdesk.convert+encode.enqueue");
    convert(slot, stream_, (stamp && devclk_) ? ts_ + slot : nullptr);
    encode_converted(force_idr);
}

void Session::encode_converted(bool force_idr) {
    enc_->submit(nv12_y_[cur_k_], nv12_uv_[cur_k_], force_idr);
    enqueue_mask_sse(cur_k_);
}

void Session::enqueue_mask_sse(int k) {
    // after the analysis kernels on stream_ (reconstruction final, source not yet overwritten
    // by the next frame's conversion, which is later on the same stream)
    if (!masked() || mask_in_encoder_) return;
    const h264::EncoderConfig& e = enc_->rc().config();
    int r[4];
    mask_rect_mb(r);
    pix::launch_sse_masked(nv12_y_[k], enc_->recon_y(), enc_->pitch(), e.width, e.height, r[0], r[1], r[2], r[3],
                           mask_dev_ + (size_t)k * mask_stride_, mask_counter_ + k, mask_host_ + k,
                           stream_);  // mapped: the kernel stores the total to the host
    HIP_CHECK(hipEventRecord(ev_mask_[k], stream_));
}

void Session::mask_rect_mb(int r[4]) const {
    // the quality mask widened to whole 16x16 macroblocks and clipped to the picture: the same
    // region the H.264 encoder leaves out of its masked distortion channel, so both codecs'
    // masked PSNR figures cover the same pixels
    const h264::EncoderConfig& e = enc_->rc().config();
    r[0] = std::max(0, cfg_.mask_x0) / 16 * 16;
    r[1] = std::max(0, cfg_.mask_y0) / 16 * 16;
    r[2] = std::min(e.width, (cfg_.mask_x1 + 15) / 16 * 16);
    r[3] = std::min(e.height, (cfg_.mask_y1 + 15) / 16 * 16);
}

int Session::begin_frame(int slot) {
    if ((int)inflight_.size() >= depth_) throw std::logic_error("Session: collect() before the next submit");
    const int k = next_k_;
    next_k_ = (next_k_ + 1) % depth_;
    inflight_.push_back(Inflight{frame_id_, now_us(), k, slot});
    t_capture_ = inflight_.back().t_capture;
    cur_k_ = last_k_ = k;
    return k;
}

pix::SynthParams Session::synth_params() {
    pix::SynthParams p;
    p.width = cfg_.width;
    p.height = cfg_.height;
    p.pitch = pool_->pitch();
    p.frame_id = frame_id_;
    p.timestamp_us = cfg_.fake_clock ? (uint32_t)((int64_t)frame_id_ * 1000000 / std::max(1, cfg_.fps))
                                     : (uint32_t)(t_capture_ - t0_us_);
    p.t = (float)frame_id_ / (float)std::max(1, cfg_.fps);
    p.origin_x = 0;
    p.origin_y = 0;
    p.wall_w = cfg_.width;
    p.wall_h = cfg_.height;
    p.noise = cfg_.noise;
    p.content = cfg_.content;
    p.cursor_x = cursor_x_;
    p.cursor_y = cursor_y_;
    return p;
}

hipGraphExec_t Session::capture_on(hipStream_t st, const std::function<void()>& body) {
    hipGraph_t graph = nullptr;
    HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    try {
        body();
        HIP_CHECK(hipGetLastError());
    } catch (...) {
        hipStreamEndCapture(st, &graph);  // leave capture mode before propagating
        if (graph) hipGraphDestroy(graph);
        throw;
    }
    HIP_CHECK(hipStreamEndCapture(st, &graph));
    hipGraphExec_t exec = nullptr;
    HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(graph));
    ++graphs_built_;
    return exec;
}

// Per-frame chain as graphs: with one frame in flight the whole chain on the session stream;
// with two, the analysis part (parameter upload, desktop render, conversion, frame-state
// upload, analysis kernels) on the session stream and the entropy part on the encoder's
// entropy stream, linked per frame by an event outside the graphs -- two graph launches and
// four event operations per frame instead of ~9 kernel launches plus those events (the host
// issue rate was the frame-rate limit: profiles/r03_h264).
void Session::capture_frame_graphs(int slot, bool idr, hipGraphExec_t* ga, hipGraphExec_t* ge) {
    TraceRange tr("mxdesk.graph.capture");
    pix::SynthParams* dev = synth_dev_ + slot;
    const pix::SynthParams* host = synth_host_ + slot;
    auto analysis = [&]() {
        HIP_CHECK(hipMemcpyAsync(dev, host, sizeof(pix::SynthParams), hipMemcpyHostToDevice, stream_));
        pix::launch_synth_dev(pool_->data(slot), dev, cfg_.width, cfg_.height, stream_, synth_bg_);
        HIP_CHECK(hipGetLastError());
        convert(slot, stream_);
    };
    if (depth_ == 1) {
        *ga = capture_on(stream_, [&]() {
            analysis();
            enc_->enqueue_body(idr, nv12_y_[cur_k_], nv12_uv_[cur_k_]);
        });
        *ge = nullptr;
        return;
    }
    *ga = capture_on(stream_, [&]() {
        analysis();
        enc_->enqueue_analysis(idr, nv12_y_[cur_k_], nv12_uv_[cur_k_]);
    });
    hipStream_t es = enc_->entropy_stream() ? enc_->entropy_stream() : stream_;
    *ge = capture_on(es, [&]() { enc_->enqueue_entropy(); });
}

void Session::submit_synthetic(bool force_idr) {
    const auto t_in = std::chrono::steady_clock::now();
    struct Acc {
        double& a;
        std::chrono::steady_clock::time_point t;
        ~Acc() { a += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count(); }
    } acc{ht_submit_, t_in};
    TraceRange tr("mxdesk.submit_synthetic");
    const int slot = pool_->acquire();
    const int k = begin_frame(slot);
    pix::SynthParams p = synth_params();
    if (devclk_) p.ts = ts_ + slot;
    ++frame_id_;
    // the first CBR frame runs eagerly: its rate-control probe encodes synchronously
    if (!cfg_.use_graph || enc_->rc().wants_probe()) {
        // capture stream: the render + conversion of this frame may run beside the previous
        // frame's analysis; the analysis stream waits only for this frame's conversion
        hipStream_t cs = cap_stream_ ? cap_stream_ : stream_;
        if (!devclk_) HIP_CHECK(hipEventRecord(ev_start_[k], cs));
        pix::launch_synth(pool_->data(slot), p, cs, synth_bg_);
        HIP_CHECK(hipGetLastError());
        TraceRange tr2("mxdesk.convert+encode.enqueue");
        convert(slot, cs);
        if (cap_stream_) {
            HIP_CHECK(hipEventRecord(ev_conv_[k], cs));
            // the encoder waits right before its first source read (or here, if it cannot)
            if (!enc_->set_input_event(ev_conv_[k])) HIP_CHECK(hipStreamWaitEvent(stream_, ev_conv_[k], 0));
        }
        encode_converted(force_idr);
        return;
    }
    enc_->quiesce();        // no helper-thread launch may land inside a capture or after a replay
    synth_host_[slot] = p;  // read by this slot's graph memcpy node (its previous frame was collected)
    const bool idr = enc_->prepare(force_idr);
    const int es = depth_ > 1 ? enc_->prep_slot() : 0;
    if (es != (depth_ > 1 ? k : 0))  // the graph bakes in the NV12 buffer of k
        throw std::logic_error("Session: encoder slot out of step with the session's frame index");
    if (!devclk_) HIP_CHECK(hipEventRecord(ev_start_[k], stream_));
    enc_->record_start();
    const size_t key = (((size_t)slot * kMaxDepth + (size_t)es) * 2 + (idr ? 1 : 0)) * 2;
    if (!graphs_[key]) capture_frame_graphs(slot, idr, &graphs_[key], &graphs_[key + 1]);
    HIP_CHECK(hipGraphLaunch(graphs_[key], stream_));
    if (graphs_[key + 1]) {
        enc_->link_entropy();
        HIP_CHECK(hipGraphLaunch(graphs_[key + 1], enc_->entropy_stream() ? enc_->entropy_stream() : stream_));
    }
    enc_->record_done();
    enqueue_mask_sse(k);
}

void Session::register_host_buffer(const void* p, size_t bytes) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (const auto& r : host_regs_)
        if (r.first == b && r.second == bytes) return;
    HIP_CHECK(hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault));
    host_regs_.emplace_back(b, bytes);
    ensure_upload_stream();
}

void Session::ensure_upload_stream() {
    if (!ev_upload_) HIP_CHECK(hipEventCreateWithFlags(&ev_upload_, hipEventDisableTiming));
    if (!upload_stream_) HIP_CHECK(hipStreamCreateWithFlags(&upload_stream_, hipStreamNonBlocking));
}

void Session::encode_uploaded(int slot, int k, bool force_idr) {
    HIP_CHECK(hipEventRecord(ev_upload_, upload_stream_));
    if (cap_stream_) {  // the conversion follows the DMA on its stream (overlaps earlier frames' analysis)
        convert(slot, upload_stream_, devclk_ ? ts_ + slot : nullptr);
        HIP_CHECK(hipEventRecord(ev_conv_[k], upload_stream_));
        HIP_CHECK(hipStreamWaitEvent(stream_, ev_conv_[k], 0));
        encode_converted(force_idr);
    } else {
        HIP_CHECK(hipStreamWaitEvent(stream_, ev_upload_, 0));
        convert_and_encode(slot, force_idr, true);  // GPU time from the conversion (DMA excluded)
    }
    HIP_CHECK(hipEventSynchronize(ev_upload_));  // the caller may overwrite the buffer now
}

void Session::submit_bgrx_damage(const uint8_t* host_bgrx, int host_pitch, size_t bytes,
                                 const std::vector<std::pair<int, int>>& bands, bool force_idr) {
    TraceRange tr("mxdesk.submit_bgrx_damage(upload)");
    if (host_pitch < cfg_.width * 4) throw std::invalid_argument("pitch < width * 4");
    const int row = cfg_.width * 4;
    const size_t span = (size_t)host_pitch * (cfg_.height - 1) + (size_t)row;
    if (host_bgrx == nullptr || bytes < span)
        throw std::invalid_argument("frame span (" + std::to_string(span) + " B) exceeds the buffer (" +
                                    std::to_string(bytes) + " B)");
    for (const auto& b : bands)
        if (b.first < 0 || b.second > cfg_.height || b.first > b.second)
            throw std::invalid_argument("damage band [" + std::to_string(b.first) + ", " + std::to_string(b.second) +
                                        ") outside the frame");
    ensure_upload_stream();
    const size_t pitch = pool_->pitch();
    if (!screen_) {
        HIP_CHECK(hipMalloc(&screen_, pitch * cfg_.height));
        screen_valid_ = false;
    }
    std::vector<std::pair<int, int>> todo;
    if (!screen_valid_) todo.emplace_back(0, cfg_.height);
    else
        for (const auto& b : bands)
            if (b.second > b.first) todo.push_back(b);
    const int slot = pool_->acquire();
    const int k = begin_frame(slot);
    ++frame_id_;
    if (!devclk_) HIP_CHECK(hipEventRecord(ev_start_[k], stream_));
    // Bands and the screen -> slot copy are ordered on the upload stream; the slot's previous
    // reader finished before its frame was collected (as in submit_bgrx's zero-copy path).
    for (const auto& b : todo) {
        HIP_CHECK(hipMemcpy2DAsync(screen_ + (size_t)b.first * pitch, pitch, host_bgrx + (size_t)b.first * host_pitch,
                                   host_pitch, row, b.second - b.first, hipMemcpyHostToDevice, upload_stream_));
        damage_bytes_ += (uint64_t)row * (b.second - b.first);
    }
    HIP_CHECK(hipMemcpyAsync(pool_->data(slot), screen_, pitch * cfg_.height, hipMemcpyDeviceToDevice,
                             upload_stream_));
    screen_valid_ = true;
    encode_uploaded(slot, k, force_idr);
}

void Session::submit_bgrx_span(const uint8_t* host_bgrx, int host_pitch, size_t bytes, bool force_idr) {
    if (host_pitch < cfg_.width * 4) throw std::invalid_argument("pitch < width * 4");
    const size_t span = (size_t)host_pitch * (cfg_.height - 1) + (size_t)cfg_.width * 4;
    if (host_bgrx == nullptr || bytes < span)
        throw std::invalid_argument("frame span (" + std::to_string(span) + " B) exceeds the buffer (" +
                                    std::to_string(bytes) + " B)");
    submit_bgrx(host_bgrx, host_pitch, force_idr);
}

void Session::submit_bgrx(const uint8_t* host_bgrx, int host_pitch, bool force_idr) {
    TraceRange tr("mxdesk.submit_bgrx(upload)");
    const int row = cfg_.width * 4;
    const size_t span = (size_t)host_pitch * (cfg_.height - 1) + row;
    for (const auto& r : host_regs_) {
        if (host_bgrx < r.first || host_bgrx + span > r.first + r.second) continue;
        // zero-copy: DMA straight from the registered capture buffer
        const int slot = pool_->acquire();
        const int k = begin_frame(slot);
        ++frame_id_;
        if (!devclk_) HIP_CHECK(hipEventRecord(ev_start_[k], stream_));
        // the DMA runs on its own stream with no dependency on stream_, so waiting for it below
        // does not also wait for the previous frames' analysis kernels queued there (keeps the
        // pipelined overlap).  The pool slot needs no ordering: its last reader (the conversion
        // pool_slots > depth frames ago) finished before that frame was collected, and a frame is
        // collected only after its whole chain completed.
        HIP_CHECK(hipMemcpy2DAsync(pool_->data(slot), pool_->pitch(), host_bgrx, host_pitch, row, cfg_.height,
                                   hipMemcpyHostToDevice, upload_stream_));
        encode_uploaded(slot, k, force_idr);
        return;
    }
    const int slot = pool_->acquire();
    const int k = begin_frame(slot);
    ++frame_id_;
    for (int r = 0; r < cfg_.height; ++r)
        std::memcpy(staging_[k] + (size_t)r * pool_->pitch(), host_bgrx + (size_t)r * host_pitch, row);
    if (!devclk_) HIP_CHECK(hipEventRecord(ev_start_[k], stream_));
    HIP_CHECK(hipMemcpyAsync(pool_->data(slot), staging_[k], (size_t)pool_->pitch() * cfg_.height,
                             hipMemcpyHostToDevice, stream_));
    convert_and_encode(slot, force_idr, true);  // GPU time from the conversion (upload excluded)
}

FrameResult Session::collect() {
    if (inflight_.empty()) throw std::logic_error("Session: nothing submitted");
    const Inflight fl = inflight_.front();
    inflight_.pop_front();
    FrameResult r;
    TraceRange tr("mxdesk.collect(wait+annexb)");
    const auto t_in = std::chrono::steady_clock::now();
    wait_event(enc_->pending_done_event());  // MXDESK_WAIT=spin polls instead of blocking
    const auto t_w = std::chrono::steady_clock::now();
    const std::vector<uint8_t>& au = enc_->collect();
    r.t_encoded_us = now_us();
    ht_wait_ += std::chrono::duration<double, std::micro>(t_w - t_in).count();
    ++ht_n_;
    struct Acc {
        double& a;
        std::chrono::steady_clock::time_point t;
        ~Acc() { a += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count(); }
    } acc{ht_post_, t_w};
    r.au = au;
    r.frame_id = fl.frame_id;
    r.t_capture_us = fl.t_capture;  // steady clock (CLOCK_MONOTONIC) microseconds
    const h264::FrameStats& st = enc_->last_stats();
    r.idr = st.idr;
    r.qp = st.qp;
    r.deblocked = st.deblocked;
    r.db_coherent = st.db_coherent;
    r.db_moving = st.db_moving;
    if (devclk_) {  // device clock: first kernel of the frame (render / conversion) -> end of its pack kernel
        const uint64_t t0 = ts_[fl.slot], t1 = enc_->last_t_end();
        r.gpu_ms = t1 > t0 ? (double)(t1 - t0) / clock_khz_ : 0.0;
    } else {  // render/upload start -> bitstream written (events)
        float ms = 0;
        hipEventElapsedTime(&ms, ev_start_[fl.k], enc_->done_event());
        r.gpu_ms = ms;
    }
    const double ny = (double)enc_->rc().config().width * enc_->rc().config().height, nc = ny / 4;
    auto psnr = [](uint64_t sse, double n) { return sse == 0 ? 99.0 : std::min(99.0, 10.0 * std::log10(65025.0 * n / (double)sse)); };
    r.psnr_y = psnr(st.sse[0], ny);
    r.psnr_u = psnr(st.sse[1], nc);
    r.psnr_v = psnr(st.sse[2], nc);
    if (masked() && mask_in_encoder_) {
        r.psnr_y_masked = psnr(st.sse_masked, (double)std::max<int64_t>(1, st.masked_pixels));
    } else if (masked()) {
        HIP_CHECK(hipEventSynchronize(ev_mask_[fl.k]));
        int m[4];
        mask_rect_mb(m);
        const double mw = std::max(0, m[2] - m[0]), mh = std::max(0, m[3] - m[1]);
        r.psnr_y_masked = psnr(mask_host_[fl.k], std::max(1.0, ny - mw * mh));
    }
    return r;
}

PacedStats run_sessions_paced(const std::vector<Session*>& sessions, int fps, double seconds, int threads,
                              int idr_slot) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    const int k = (int)sessions.size();
    threads = std::max(1, std::min(threads, k));
    const int slots = std::max(1, (int)std::lround(seconds * fps));
    const auto period = std::chrono::nanoseconds((int64_t)(1e9 / std::max(1, fps)));
    std::vector<std::vector<uint8_t>> late(threads, std::vector<uint8_t>(slots, 0));
    std::vector<std::vector<double>> lat(threads), idr_lat(threads);
    std::vector<std::exception_ptr> err(threads);
    // every thread starts on the same slot grid (a little ahead, so all are waiting for slot 0)
    const auto t0 = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        th.emplace_back([&, t]() {
            try {
                HIP_CHECK(hipSetDevice(dev));
                std::vector<Session*> mine;
                for (int i = t; i < k; i += threads) mine.push_back(sessions[i]);
                lat[t].reserve(mine.size() * (size_t)slots);
                for (int f = 0; f < slots; ++f) {
                    const auto tick = t0 + f * period;
                    std::this_thread::sleep_until(tick);
                    const bool storm = f == idr_slot;  // every session's key frame in one slot
                    for (Session* s : mine) s->submit_synthetic(storm);
                    for (Session* s : mine) {
                        const FrameResult r = s->collect();
                        const double ms = (r.t_encoded_us - r.t_capture_us) / 1000.0;
                        lat[t].push_back(ms);
                        if (storm) idr_lat[t].push_back(ms);
                    }
                    late[t][f] = std::chrono::steady_clock::now() > tick + period ? 1 : 0;
                }
            } catch (...) {
                err[t] = std::current_exception();
            }
        });
    }
    for (auto& x : th) x.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    PacedStats st;
    st.slots = slots;
    for (int f = 0; f < slots; ++f) {
        bool l = false;
        for (int t = 0; t < threads; ++t) l |= late[t][f] != 0;
        st.late_slots += l ? 1 : 0;
    }
    for (auto& v : lat) st.lat_ms.insert(st.lat_ms.end(), v.begin(), v.end());
    for (auto& v : idr_lat) st.idr_lat_ms.insert(st.idr_lat_ms.end(), v.begin(), v.end());
    if (idr_slot >= 0 && idr_slot < slots)
        for (int t = 0; t < threads; ++t) st.idr_late |= late[t][idr_slot] != 0;
    return st;
}

std::vector<std::vector<FrameResult>> run_sessions(const std::vector<Session*>& sessions, int n_frames, int depth) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    const size_t k = sessions.size();
    std::vector<std::vector<FrameResult>> out(k);
    std::vector<std::exception_ptr> err(k);
    std::vector<std::thread> th;
    th.reserve(k);
    auto drive = [&](size_t i) {
            try {
                HIP_CHECK(hipSetDevice(dev));
                Session& s = *sessions[i];
                const int d = std::max(1, std::min(depth, s.depth()));
                out[i].reserve((size_t)n_frames);
                int sent = 0;
                while (sent < std::min(d, n_frames)) {
                    s.submit_synthetic(false);
                    ++sent;
                }
                for (int f = 0; f < n_frames; ++f) {
                    out[i].push_back(s.collect());
                    if (sent < n_frames) {
                        s.submit_synthetic(false);
                        ++sent;
                    }
                }
            } catch (...) {
                err[i] = std::current_exception();
            }
    };
    // one session runs on the calling thread (no thread start-up inside a caller's timed region)
    if (k == 1) {
        drive(0);
    } else {
        for (size_t i = 0; i < k; ++i) th.emplace_back(drive, i);
        for (auto& t : th) t.join();
    }
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    return out;
}

}  // namespace mx
