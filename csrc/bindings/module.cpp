// pybind11 bindings: mxdesk._native
// Device buffers are passed as integer pointers (e.g. torch.Tensor.data_ptr()) and HIP
// streams as integers (torch.cuda.current_stream().cuda_stream), so the kernels compose
// with PyTorch-ROCm tensors and torch.distributed (RCCL) without copies.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../codec/h264_core.h"
#include "../codec/h264_encoder.h"
#include "../codec/vp8_encoder.h"
#include "../codec/hevc_encoder.h"
#include "../common/hip_check.h"
#include "../common/trace.h"
#include "../kernels/pixel.h"
#include "../runtime/session.h"

namespace py = pybind11;
using namespace mx;

void register_net(py::module& m);    // net_bindings.cpp
void register_audio(py::module& m);  // audio_bindings.cpp
void register_rfb(py::module& m);    // rfb_bindings.cpp

namespace {

template <class T>
T* as_ptr(uintptr_t p) {
    return reinterpret_cast<T*>(p);
}
hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::bytes to_bytes(const std::vector<uint8_t>& v) {
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

// --- bit helpers exposed for unit tests
struct PyBits {
    std::vector<uint32_t> words;
    h264::BitWriter w;
    PyBits() : words(4096) { w.init(words.data()); }
    py::tuple finish() {
        const uint32_t bits = w.bits;
        w.flush();
        std::vector<uint8_t> out;
        for (uint32_t i = 0; i < (bits + 7) / 8; ++i) out.push_back((uint8_t)(words[i / 4] >> (24 - 8 * (i % 4))));
        return py::make_tuple(to_bytes(out), bits);
    }
};

py::tuple cavlc_block_py(const std::vector<int>& coef, int nc) {
    PyBits b;
    int16_t c[16] = {0};
    const int n = (int)coef.size();
    if (n != 4 && n != 15 && n != 16) throw std::invalid_argument("block must have 4, 15 or 16 coefficients");
    for (int i = 0; i < n; ++i) c[i] = (int16_t)coef[i];
    h264::cavlc_block(b.w, c, n, nc);
    return b.finish();
}

py::array_t<int> fdct_py(py::array_t<int, py::array::c_style | py::array::forcecast> x) {
    if (x.size() != 16) throw std::invalid_argument("need 16 values");
    py::array_t<int> y(16);
    h264::fdct4x4(x.data(), y.mutable_data());
    return y;
}
py::array_t<int> idct_py(py::array_t<int, py::array::c_style | py::array::forcecast> x) {
    if (x.size() != 16) throw std::invalid_argument("need 16 values");
    py::array_t<int> y(16);
    h264::idct4x4(x.data(), y.mutable_data());
    return y;
}

py::array_t<uint8_t> copy_plane(const uint8_t* dev, int pitch, int w, int h) {
    py::array_t<uint8_t> out({h, w});
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipMemcpy2D(out.mutable_data(), w, dev, pitch, w, h, hipMemcpyDeviceToHost));
    return out;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
    m.doc() = "mxdesk native runtime: HIP kernels (gfx950), H.264 encoder, session pipeline";

    m.def("device_count", []() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) return 0;
        return n;
    });
    m.def("set_device", [](int d) { HIP_CHECK(hipSetDevice(d)); });
    m.def("device_name", [](int d) {
        hipDeviceProp_t p;
        HIP_CHECK(hipGetDeviceProperties(&p, d));
        return std::string(p.gcnArchName) + " / " + p.name;
    });
    m.def("synchronize", []() { HIP_CHECK(hipDeviceSynchronize()); });
    register_net(m);
    register_audio(m);
    register_rfb(m);
    m.def("now_us", &Session::now_us, "CLOCK_MONOTONIC microseconds (same clock as time.monotonic())");

    // ---------------------------------------------------------------- codec helpers
    py::module h = m.def_submodule("h264", "H.264 building blocks (for tests)");
    h.def("hpel_planes", [](py::array_t<uint8_t, py::array::c_style> ref, int coded_w) {
        if (ref.ndim() != 2 || coded_w % 16 || ref.shape(0) % 16 || ref.shape(1) < coded_w)
            throw std::invalid_argument("ref must be (coded_h, pitch) with 16-aligned coded size");
        int hp = 0;
        auto planes = h264::hpel_planes_for_test(ref.data(), coded_w, (int)ref.shape(0), (int)ref.shape(1), &hp);
        const int rows = (int)ref.shape(0) + 2 * h264::kHpelPad;
        py::list out;
        for (auto& p : planes) {
            py::array_t<uint8_t> a({rows, hp});
            std::memcpy(a.mutable_data(), p.data(), p.size());
            out.append(a);
        }
        return out;
    });
    h.def("cavlc_block", &cavlc_block_py, py::arg("coef"), py::arg("nc"));
    h.def("fdct4x4", &fdct_py);
    h.def("idct4x4", &idct_py);
    h.def("ue", [](uint32_t k) {
        PyBits b;
        h264::put_ue(b.w, k);
        return b.finish();
    });
    h.def("se", [](int v) {
        PyBits b;
        h264::put_se(b.w, v);
        return b.finish();
    });
    h.def("luma_qpel", [](py::array_t<uint8_t, py::array::c_style> plane, int x4, int y4) {
        if (plane.ndim() != 2) throw std::invalid_argument("2-D plane");
        const int H = (int)plane.shape(0), W = (int)plane.shape(1);
        return h264::luma_qpel(plane.data(), W, W, H, x4, y4);
    });
    h.def("level_for", &h264::pick_level);

    py::class_<h264::EncoderConfig>(m, "EncoderConfig")
        .def(py::init<>())
        .def_readwrite("width", &h264::EncoderConfig::width)
        .def_readwrite("height", &h264::EncoderConfig::height)
        .def_readwrite("fps", &h264::EncoderConfig::fps)
        .def_readwrite("bitrate_kbps", &h264::EncoderConfig::bitrate_kbps)
        .def_readwrite("qp", &h264::EncoderConfig::qp)
        .def_readwrite("qp_min", &h264::EncoderConfig::qp_min)
        .def_readwrite("qp_max", &h264::EncoderConfig::qp_max)
        .def_readwrite("keyint", &h264::EncoderConfig::keyint)
        .def_readwrite("search_range", &h264::EncoderConfig::search_range)
        .def_readwrite("me_coarse", &h264::EncoderConfig::me_coarse)
        .def_readwrite("intra4x4", &h264::EncoderConfig::intra4x4)
        .def_readwrite("subpel", &h264::EncoderConfig::subpel)
        .def_readwrite("chroma_qp_offset", &h264::EncoderConfig::chroma_qp_offset)
        .def_readwrite("pipeline_depth", &h264::EncoderConfig::pipeline_depth)
        .def_readwrite("aq", &h264::EncoderConfig::aq)
        .def_readwrite("intra_in_p", &h264::EncoderConfig::intra_in_p)
        .def_readwrite("vp8_bpred", &h264::EncoderConfig::vp8_bpred)
        .def_readwrite("vp8_intra", &h264::EncoderConfig::vp8_intra)
        .def_readwrite("mask_x0", &h264::EncoderConfig::mask_x0)
        .def_readwrite("mask_y0", &h264::EncoderConfig::mask_y0)
        .def_readwrite("mask_x1", &h264::EncoderConfig::mask_x1)
        .def_readwrite("mask_y1", &h264::EncoderConfig::mask_y1)
        .def_readwrite("deblock", &h264::EncoderConfig::deblock)
        .def_readwrite("partitions", &h264::EncoderConfig::partitions)
        .def_readwrite("tu_split", &h264::EncoderConfig::tu_split)
        .def_readwrite("hevc_slice_cost", &h264::EncoderConfig::hevc_slice_cost)
        .def_readwrite("hevc_wpp", &h264::EncoderConfig::hevc_wpp)
        .def_readwrite("hevc_wpp_rows", &h264::EncoderConfig::hevc_wpp_rows)
        .def_readwrite("sao", &h264::EncoderConfig::sao)
        .def_readwrite("hevc_chroma_keep", &h264::EncoderConfig::hevc_chroma_keep)
        .def_readwrite("hevc_intra_split", &h264::EncoderConfig::hevc_intra_split);

    py::class_<h264::FrameStats>(m, "FrameStats")
        .def_readonly("frame_index", &h264::FrameStats::frame_index)
        .def_readonly("idr", &h264::FrameStats::idr)
        .def_readonly("qp", &h264::FrameStats::qp)
        .def_readonly("bytes", &h264::FrameStats::bytes)
        .def_readonly("skipped_mbs", &h264::FrameStats::skipped_mbs)
        .def_readonly("encode_ms", &h264::FrameStats::encode_ms)
        .def_property_readonly("sse", [](const h264::FrameStats& s) { return py::make_tuple(s.sse[0], s.sse[1], s.sse[2]); })
        .def_readonly("sse_masked", &h264::FrameStats::sse_masked)
        .def_readonly("masked_pixels", &h264::FrameStats::masked_pixels)
        .def_readonly("deblocked", &h264::FrameStats::deblocked)
        .def_readonly("db_coherent", &h264::FrameStats::db_coherent)
        .def_readonly("db_changed", &h264::FrameStats::db_changed)
        .def_readonly("db_moving", &h264::FrameStats::db_moving);

    py::class_<h264::CpuH264Encoder>(m, "CpuH264Encoder")
        .def(py::init<const h264::EncoderConfig&>())
        .def(
            "encode",
            [](h264::CpuH264Encoder& e, py::array_t<uint8_t, py::array::c_style> y,
               py::array_t<uint8_t, py::array::c_style> uv, bool force_idr) {
                if (y.ndim() != 2 || uv.ndim() != 2 || y.shape(1) != uv.shape(1))
                    throw std::invalid_argument("y (H,P) and uv (H/2,P) planes with equal pitch");
                const int pitch = (int)y.shape(1);
                const int cw = e.coded_pitch();
                const auto& cfg = e.common().config();
                const int ch = e.common().mb_h() * 16;
                if (y.shape(0) < cfg.height || pitch < cfg.width || uv.shape(0) < cfg.height / 2)
                    throw std::invalid_argument("planes smaller than the encoder's configured picture");
                std::vector<uint8_t> py_, puv;
                const uint8_t* yy = y.data();
                const uint8_t* uu = uv.data();
                int p = pitch;
                if (y.shape(0) < ch || pitch < cw) {
                    h264::pad_nv12(yy, uu, cfg.width, cfg.height, pitch, cw, ch, py_, puv);
                    yy = py_.data();
                    uu = puv.data();
                    p = cw;
                }
                const auto& au = e.encode(yy, uu, p, force_idr);
                return to_bytes(au);
            },
            py::arg("y"), py::arg("uv"), py::arg("force_idr") = false)
        .def("recon",
             [](h264::CpuH264Encoder& e) {
                 const int cw = e.coded_pitch(), ch = e.common().mb_h() * 16;
                 py::array_t<uint8_t> y({ch, cw}), uv({ch / 2, cw});
                 std::memcpy(y.mutable_data(), e.recon_y().data(), (size_t)cw * ch);
                 std::memcpy(uv.mutable_data(), e.recon_uv().data(), (size_t)cw * ch / 2);
                 return py::make_tuple(y, uv);
             })
        .def("mb_bits",
             [](h264::CpuH264Encoder& e) {
                 const auto& v = e.mb_bits();
                 py::array_t<uint32_t> a((py::ssize_t)v.size());
                 std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
                 return a.reshape({e.common().mb_h(), e.common().mb_w()});
             })
        .def("mb_info",
             [](h264::CpuH264Encoder& e) {  // (mb_h, mb_w, 9): type, qp, cbp, skip, mvx, mvy, nz_luma sum, cost, part
                 const auto& v = e.mb_info();
                 py::array_t<int32_t> a({(py::ssize_t)v.size(), (py::ssize_t)9});
                 int32_t* d = a.mutable_data();
                 for (size_t i = 0; i < v.size(); ++i) {
                     int nz = 0;
                     for (int k = 0; k < 16; ++k) nz += v[i].nz_luma[k];
                     const int32_t r[9] = {v[i].type, v[i].qp, v[i].cbp, v[i].skip, v[i].mvx, v[i].mvy, nz,
                                           (int32_t)v[i].cost, v[i].part};
                     std::memcpy(d + 9 * i, r, sizeof r);
                 }
                 return a.reshape({e.common().mb_h(), e.common().mb_w(), 9});
             })
        .def("request_idr", [](h264::CpuH264Encoder& e) { e.common().request_idr(); })
        .def("set_bitrate", [](h264::CpuH264Encoder& e, int k) { e.common().set_bitrate(k); })
        .def_property_readonly("stats", &h264::CpuH264Encoder::last_stats);

    py::class_<vp8::CpuVp8Encoder>(m, "CpuVp8Encoder")
        .def(py::init<const h264::EncoderConfig&>())
        .def(
            "encode",
            [](vp8::CpuVp8Encoder& e, py::array_t<uint8_t, py::array::c_style> y,
               py::array_t<uint8_t, py::array::c_style> uv, bool force_idr) {
                if (y.ndim() != 2 || uv.ndim() != 2 || y.shape(1) != uv.shape(1))
                    throw std::invalid_argument("y (H,P) and uv (H/2,P) planes with equal pitch");
                const int pitch = (int)y.shape(1);
                const int cw = e.coded_pitch();
                const auto& cfg = e.common().config();
                const int ch = e.common().mb_h() * 16;
                if (y.shape(0) < cfg.height || pitch < cfg.width || uv.shape(0) < cfg.height / 2)
                    throw std::invalid_argument("planes smaller than the encoder's configured picture");
                std::vector<uint8_t> py_, puv;
                const uint8_t* yy = y.data();
                const uint8_t* uu = uv.data();
                int p = pitch;
                if (y.shape(0) < ch || pitch < cw) {
                    h264::pad_nv12(yy, uu, cfg.width, cfg.height, pitch, cw, ch, py_, puv);
                    yy = py_.data();
                    uu = puv.data();
                    p = cw;
                }
                const auto& au = e.encode(yy, uu, p, force_idr);
                return to_bytes(au);
            },
            py::arg("y"), py::arg("uv"), py::arg("force_idr") = false)
        .def("recon",
             [](vp8::CpuVp8Encoder& e) {
                 const int cw = e.coded_pitch(), ch = e.common().mb_h() * 16;
                 py::array_t<uint8_t> y({ch, cw}), uv({ch / 2, cw});
                 std::memcpy(y.mutable_data(), e.recon_y().data(), (size_t)cw * ch);
                 std::memcpy(uv.mutable_data(), e.recon_uv().data(), (size_t)cw * ch / 2);
                 return py::make_tuple(y, uv);
             })
        .def("mb_info",
             [](vp8::CpuVp8Encoder& e) {  // (nmb, 4): ymode, uvmode, mvx, mvy (1/8 samples)
                 const auto& v = e.mb_info();
                 py::array_t<int32_t> a({(py::ssize_t)v.size(), (py::ssize_t)4});
                 int32_t* d = a.mutable_data();
                 for (size_t i = 0; i < v.size(); ++i) {
                     d[4 * i] = v[i].ymode;
                     d[4 * i + 1] = v[i].uvmode;
                     d[4 * i + 2] = v[i].mvx;
                     d[4 * i + 3] = v[i].mvy;
                 }
                 return a;
             })
        .def("request_idr", [](vp8::CpuVp8Encoder& e) { e.common().request_idr(); })
        .def("set_bitrate", [](vp8::CpuVp8Encoder& e, int k) { e.common().set_bitrate(k); })
        .def_property_readonly("stats", &vp8::CpuVp8Encoder::last_stats)
        .def_property_readonly("writer_first_us", &vp8::CpuVp8Encoder::writer_first_us)
        .def_property_readonly("writer_tokens_us", &vp8::CpuVp8Encoder::writer_tokens_us);

    py::class_<vp8::GpuVp8Encoder>(m, "GpuVp8Encoder")
        .def(py::init([](const h264::EncoderConfig& c, uintptr_t stream) {
                 return new vp8::GpuVp8Encoder(c, as_stream(stream));
             }),
             py::arg("config"), py::arg("stream") = 0)
        .def_property_readonly("pitch", &vp8::GpuVp8Encoder::pitch)
        .def_property_readonly("coded_height", [](vp8::GpuVp8Encoder& e) { return e.geometry().coded_h; })
        .def(
            "encode",
            [](vp8::GpuVp8Encoder& e, uintptr_t y, uintptr_t uv, bool force_idr) {
                std::vector<uint8_t> au;
                {
                    py::gil_scoped_release rel;
                    e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr);
                    au = e.collect();
                }
                return to_bytes(au);
            },
            py::arg("y_ptr"), py::arg("uv_ptr"), py::arg("force_idr") = false)
        .def("submit", [](vp8::GpuVp8Encoder& e, uintptr_t y, uintptr_t uv,
                          bool force_idr) { e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr); })
        .def("collect",
             [](vp8::GpuVp8Encoder& e) {
                 std::vector<uint8_t> au;
                 {
                     py::gil_scoped_release rel;
                     au = e.collect();
                 }
                 return to_bytes(au);
             })
        .def("recon",
             [](vp8::GpuVp8Encoder& e) {
                 const auto& g = e.geometry();
                 return py::make_tuple(copy_plane(e.recon_y(), g.pitch, g.coded_w, g.coded_h),
                                       copy_plane(e.recon_uv(), g.pitch, g.coded_w, g.coded_h / 2));
             })
        .def("mb_info",
             [](vp8::GpuVp8Encoder& e) {  // (nmb, 4) of the last collected frame, as CpuVp8Encoder.mb_info
                 const auto& g = e.geometry();
                 const size_t n = (size_t)g.mb_w * g.mb_h;
                 py::array_t<int32_t> a({(py::ssize_t)n, (py::ssize_t)4});
                 int32_t* d = a.mutable_data();
                 const vp8::Vp8Mb* v = e.last_mb_info();
                 if (!v) throw std::logic_error("GpuVp8Encoder: no frame collected");
                 for (size_t i = 0; i < n; ++i) {
                     d[4 * i] = v[i].ymode;
                     d[4 * i + 1] = v[i].uvmode;
                     d[4 * i + 2] = v[i].mvx;
                     d[4 * i + 3] = v[i].mvy;
                 }
                 return a;
             })
        .def("request_idr", [](vp8::GpuVp8Encoder& e) { e.common().request_idr(); })
        .def("set_bitrate", [](vp8::GpuVp8Encoder& e, int k) { e.common().set_bitrate(k); })
        .def_property_readonly("stats", &vp8::GpuVp8Encoder::last_stats);

    m.def("hevc_token_selftest", &hevc::token_selftest, py::arg("seed"), py::arg("slices"));
    py::class_<hevc::CpuHevcEncoder>(m, "CpuHevcEncoder")
        .def(py::init<const h264::EncoderConfig&>())
        .def(
            "encode",
            [](hevc::CpuHevcEncoder& e, py::array_t<uint8_t, py::array::c_style> y,
               py::array_t<uint8_t, py::array::c_style> uv, bool force_idr) {
                if (y.ndim() != 2 || uv.ndim() != 2 || y.shape(1) != uv.shape(1))
                    throw std::invalid_argument("y (H,P) and uv (H/2,P) planes with equal pitch");
                const int pitch = (int)y.shape(1);
                const int cw = e.coded_pitch();
                const auto& cfg = e.common().config();
                const int ch = e.common().ctb_h() * hevc::kCtb;
                std::vector<uint8_t> py_, puv;
                const uint8_t* yy = y.data();
                const uint8_t* uu = uv.data();
                int p = pitch;
                if (y.shape(0) < ch || pitch < cw) {
                    h264::pad_nv12(yy, uu, cfg.width, cfg.height, pitch, cw, ch, py_, puv);
                    yy = py_.data();
                    uu = puv.data();
                    p = cw;
                }
                std::vector<uint8_t> au;
                {
                    py::gil_scoped_release rel;
                    au = e.encode(yy, uu, p, force_idr);
                }
                return to_bytes(au);
            },
            py::arg("y"), py::arg("uv"), py::arg("force_idr") = false)
        .def("recon",
             [](hevc::CpuHevcEncoder& e) {
                 const int cw = e.coded_pitch(), ch = e.common().ctb_h() * hevc::kCtb;
                 py::array_t<uint8_t> y({ch, cw}), uv({ch / 2, cw});
                 std::memcpy(y.mutable_data(), e.recon_y().data(), (size_t)cw * ch);
                 std::memcpy(uv.mutable_data(), e.recon_uv().data(), (size_t)cw * ch / 2);
                 return py::make_tuple(y, uv);
             })
        .def("cu_types",
             [](hevc::CpuHevcEncoder& e) {
                 std::vector<int> t;
                 for (const auto& c : e.cus()) t.push_back(c.type);
                 return t;
             })
        .def("cu_info",  // (type, qp, cbf, tu_split, coding-tree depth, 4x4 luma node mask) per 16x16 unit
             [](hevc::CpuHevcEncoder& e) {
                 const auto& cus = e.cus();
                 py::array_t<int32_t> a({(py::ssize_t)cus.size(), (py::ssize_t)6});
                 auto m = a.mutable_unchecked<2>();
                 for (size_t i = 0; i < cus.size(); ++i) {
                     m(i, 0) = cus[i].type;
                     m(i, 1) = cus[i].qp;
                     m(i, 2) = cus[i].cbf;
                     m(i, 3) = cus[i].tu_split;
                     m(i, 4) = cus[i].ct;
                     m(i, 5) = cus[i].tu4;
                 }
                 return a;
             })
        .def_property_readonly("slice_rows", [](hevc::CpuHevcEncoder& e) { return e.common().slice_rows(); })
        .def_property_readonly("level_idc", [](hevc::CpuHevcEncoder& e) { return e.common().level_idc(); })
        .def("request_idr", [](hevc::CpuHevcEncoder& e) { e.common().rc().request_idr(); })
        .def("set_bitrate", [](hevc::CpuHevcEncoder& e, int k) { e.common().rc().set_bitrate(k); })
        .def_property_readonly("stats", &hevc::CpuHevcEncoder::last_stats);
    py::class_<hevc::GpuHevcEncoder>(m, "GpuHevcEncoder")
        .def(py::init([](const h264::EncoderConfig& c, uintptr_t stream) {
                 return new hevc::GpuHevcEncoder(c, as_stream(stream));
             }),
             py::arg("config"), py::arg("stream") = 0)
        .def_property_readonly("pitch", &hevc::GpuHevcEncoder::pitch)
        .def_property_readonly("coded_height", [](hevc::GpuHevcEncoder& e) { return e.geometry().coded_h; })
        .def_property_readonly("slice_rows", [](hevc::GpuHevcEncoder& e) { return e.common().slice_rows(); })
        .def(
            "encode",
            [](hevc::GpuHevcEncoder& e, uintptr_t y, uintptr_t uv, bool force_idr) {
                std::vector<uint8_t> au;
                {
                    py::gil_scoped_release rel;
                    e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr);
                    au = e.collect();
                }
                return to_bytes(au);
            },
            py::arg("y_ptr"), py::arg("uv_ptr"), py::arg("force_idr") = false)
        .def("submit", [](hevc::GpuHevcEncoder& e, uintptr_t y, uintptr_t uv,
                          bool force_idr) { e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr); })
        .def("collect",
             [](hevc::GpuHevcEncoder& e) {
                 std::vector<uint8_t> au;
                 {
                     py::gil_scoped_release rel;
                     au = e.collect();
                 }
                 return to_bytes(au);
             })
        .def("recon",
             [](hevc::GpuHevcEncoder& e) {
                 const auto& g = e.geometry();
                 return py::make_tuple(copy_plane(e.recon_y(), g.pitch, g.coded_w, g.coded_h),
                                       copy_plane(e.recon_uv(), g.pitch, g.coded_w, g.coded_h / 2));
             })
        .def("slice_timing", &hevc::GpuHevcEncoder::slice_timing)
        .def("request_idr", [](hevc::GpuHevcEncoder& e) { e.common().rc().request_idr(); })
        .def("set_bitrate", [](hevc::GpuHevcEncoder& e, int k) { e.common().rc().set_bitrate(k); })
        .def_property_readonly("stats", &hevc::GpuHevcEncoder::last_stats);
    m.def("hevc_level", &hevc::pick_level, py::arg("width"), py::arg("height"), py::arg("fps"));
    // Test hook: the VP8 boolean encoder (vp8_encoder.h BoolEncoder) over (probability, bit)
    // pairs, flushed -- checked against the RFC 6386 per-bit form in tests/test_vp8_bool.py
    m.def(
        "vp8_bool_encode",
        [](py::array_t<int32_t, py::array::c_style> probs, py::array_t<int32_t, py::array::c_style> bits) {
            if (probs.size() != bits.size()) throw std::invalid_argument("probs and bits differ in length");
            std::vector<uint8_t> out;
            vp8::BoolEncoder e(out);
            const int32_t* p = probs.data();
            const int32_t* b = bits.data();
            for (py::ssize_t i = 0; i < probs.size(); ++i) {
                if (p[i] < 1 || p[i] > 255) throw std::invalid_argument("probability outside 1..255");
                e.put(p[i], b[i] != 0);
            }
            e.flush();
            return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
        },
        py::arg("probs"), py::arg("bits"));

    py::class_<h264::GpuH264Encoder>(m, "GpuH264Encoder")
        .def(py::init([](const h264::EncoderConfig& c, uintptr_t stream) {
                 return new h264::GpuH264Encoder(c, as_stream(stream));
             }),
             py::arg("config"), py::arg("stream") = 0)
        .def_property_readonly("pitch", &h264::GpuH264Encoder::pitch)
        .def_property_readonly("coded_height", [](h264::GpuH264Encoder& e) { return e.geometry().coded_h; })
        .def(
            "encode",
            [](h264::GpuH264Encoder& e, uintptr_t y, uintptr_t uv, bool force_idr) {
                {
                    py::gil_scoped_release rel;
                    e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr);
                }
                std::vector<uint8_t> au;
                {
                    py::gil_scoped_release rel;
                    au = e.collect();
                }
                return to_bytes(au);
            },
            py::arg("y_ptr"), py::arg("uv_ptr"), py::arg("force_idr") = false)
        .def("submit", [](h264::GpuH264Encoder& e, uintptr_t y, uintptr_t uv,
                          bool force_idr) { e.submit(as_ptr<const uint8_t>(y), as_ptr<const uint8_t>(uv), force_idr); })
        .def("collect",
             [](h264::GpuH264Encoder& e) {
                 std::vector<uint8_t> au;
                 {
                     py::gil_scoped_release rel;
                     au = e.collect();
                 }
                 return to_bytes(au);
             })
        .def("recon",
             [](h264::GpuH264Encoder& e) {
                 const auto& g = e.geometry();
                 return py::make_tuple(copy_plane(e.recon_y(), g.pitch, g.coded_w, g.coded_h),
                                       copy_plane(e.recon_uv(), g.pitch, g.coded_w, g.coded_h / 2));
             })
        .def("request_idr", [](h264::GpuH264Encoder& e) { e.common().request_idr(); })
        .def("set_bitrate", [](h264::GpuH264Encoder& e, int k) { e.common().set_bitrate(k); })
        .def_property_readonly("stats", &h264::GpuH264Encoder::last_stats);

    // ---------------------------------------------------------------- pixel kernels
    // roctx ranges from Python (packetize / send stages of the streaming pipeline)
    m.def("h264_deblock_row_stamps", &h264::deblock_row_stamps, py::arg("mb_h"),
          "device wall-clock (start, end) of each k_deblock row wave of the last picture: luma rows, then chroma");
    m.def("device_clock_khz", &device_clock_khz);
    m.def("trace_push", [](const std::string& name) { roctxRangePushA(name.c_str()); });
    m.def("trace_pop", []() { roctxRangePop(); });
    m.def("trace_mark", [](const std::string& name) { roctxMarkA(name.c_str()); });
    m.def(
        "synth",
        [](uintptr_t out, int w, int h, int pitch, uint32_t frame_id, uint32_t ts, float t, int noise, int ox, int oy,
           int wall_w, int wall_h, int cx, int cy, uintptr_t stream, uintptr_t static_bg, int content) {
            pix::SynthParams p{w, h, pitch, frame_id, ts, t, ox, oy, wall_w > 0 ? wall_w : w, wall_h > 0 ? wall_h : h,
                               noise, cx, cy};
            p.content = content;
            pix::launch_synth(as_ptr<uint8_t>(out), p, as_stream(stream), as_ptr<const uint8_t>(static_bg));
            HIP_CHECK(hipGetLastError());
        },
        py::arg("out_ptr"), py::arg("width"), py::arg("height"), py::arg("pitch"), py::arg("frame_id") = 0,
        py::arg("timestamp_us") = 0, py::arg("t") = 0.f, py::arg("noise") = 1, py::arg("origin_x") = 0,
        py::arg("origin_y") = 0, py::arg("wall_w") = 0, py::arg("wall_h") = 0, py::arg("cursor_x") = -1,
        py::arg("cursor_y") = -1, py::arg("stream") = 0, py::arg("static_bg") = 0, py::arg("content") = 0);
    m.def(
        "composite_nv12",
        [](uintptr_t tiles, int tw, int th, int cols, int rows, uintptr_t y, uintptr_t uv, int pitch,
           uintptr_t stream) {
            pix::launch_composite_nv12(as_ptr<const uint8_t>(tiles), tw, th, cols, rows, as_ptr<uint8_t>(y),
                                       as_ptr<uint8_t>(uv), pitch, as_stream(stream));
            HIP_CHECK(hipGetLastError());
        },
        py::arg("tiles_ptr"), py::arg("tile_w"), py::arg("tile_h"), py::arg("cols"), py::arg("rows"), py::arg("y_ptr"),
        py::arg("uv_ptr"), py::arg("pitch"), py::arg("stream") = 0);
    m.def(
        "synth_static",
        [](uintptr_t out, int w, int h, int pitch, uintptr_t stream) {
            pix::SynthParams p{w, h, pitch, 0, 0, 0.f, 0, 0, w, h, 1, -1, -1};
            pix::launch_synth_static(as_ptr<uint8_t>(out), p, as_stream(stream));
            HIP_CHECK(hipGetLastError());
        },
        py::arg("out_ptr"), py::arg("width"), py::arg("height"), py::arg("pitch"), py::arg("stream") = 0);
    m.def(
        "bgrx_to_nv12",
        [](uintptr_t in, int in_pitch, int w, int h, uintptr_t y, uintptr_t uv, int out_pitch, int cw, int ch,
           uintptr_t stream) {
            if ((w & 1) || (h & 1) || (cw & 3) || (ch & 1) || cw < w || ch < h || out_pitch < cw || (out_pitch & 3) ||
                (in_pitch & 15))
                throw std::invalid_argument("bgrx_to_nv12: bad geometry");
            pix::launch_bgrx_to_nv12(as_ptr<const uint8_t>(in), in_pitch, w, h, as_ptr<uint8_t>(y), as_ptr<uint8_t>(uv),
                                     out_pitch, cw, ch, as_stream(stream));
            HIP_CHECK(hipGetLastError());
        },
        py::arg("in_ptr"), py::arg("in_pitch"), py::arg("width"), py::arg("height"), py::arg("y_ptr"),
        py::arg("uv_ptr"), py::arg("out_pitch"), py::arg("coded_w"), py::arg("coded_h"), py::arg("stream") = 0);
    m.def(
        "scale_to_nv12",
        [](uintptr_t in, int in_pitch, int in_w, int in_h, int out_w, int out_h, uintptr_t x0, uintptr_t wx, int taps_x,
           uintptr_t y0, uintptr_t wy, int taps_y, uintptr_t y, uintptr_t uv, int out_pitch, int cw, int ch,
           uintptr_t stream, bool mfma, bool strip) {
            if ((out_w & 1) || (out_h & 1) || cw < out_w || ch < out_h || (cw & 1) || (ch & 1))
                throw std::invalid_argument("scale_to_nv12: bad geometry");
            pix::LanczosTables t{out_w,
                                 out_h,
                                 taps_x,
                                 taps_y,
                                 as_ptr<const int>(x0),
                                 as_ptr<const float>(wx),
                                 as_ptr<const int>(y0),
                                 as_ptr<const float>(wy)};
            void* frags = nullptr;
            if (mfma) {  // test path: tables back to the host, fragments built and uploaded per call
                std::vector<int> hx0(out_w), hy0(out_h);
                std::vector<float> hwx((size_t)out_w * taps_x), hwy((size_t)out_h * taps_y);
                HIP_CHECK(hipMemcpy(hx0.data(), t.x0, hx0.size() * 4, hipMemcpyDeviceToHost));
                HIP_CHECK(hipMemcpy(hy0.data(), t.y0, hy0.size() * 4, hipMemcpyDeviceToHost));
                HIP_CHECK(hipMemcpy(hwx.data(), t.wx, hwx.size() * 4, hipMemcpyDeviceToHost));
                HIP_CHECK(hipMemcpy(hwy.data(), t.wy, hwy.size() * 4, hipMemcpyDeviceToHost));
                pix::ScaleFragsHost fr;
                if (!pix::build_scale_frags(in_w, in_h, out_w, out_h, cw, ch, hx0, hwx, taps_x, hy0, hwy, taps_y, fr))
                    throw std::invalid_argument("scale_to_nv12: scale factor outside the MFMA kernel's range");
                pix::upload_scale_frags(fr, &frags, t.mf);
                t.mf.force_strip = strip;  // else the one-tile-per-workgroup MFMA kernel
            }
            pix::launch_scale_to_nv12(as_ptr<const uint8_t>(in), in_pitch, in_w, in_h, t, as_ptr<uint8_t>(y),
                                      as_ptr<uint8_t>(uv), out_pitch, cw, ch, as_stream(stream));
            HIP_CHECK(hipGetLastError());
            if (frags) {
                HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
                HIP_CHECK(hipFree(frags));
            }
        },
        py::arg("in_ptr"), py::arg("in_pitch"), py::arg("in_w"), py::arg("in_h"), py::arg("out_w"), py::arg("out_h"),
        py::arg("x0_ptr"), py::arg("wx_ptr"), py::arg("taps_x"), py::arg("y0_ptr"), py::arg("wy_ptr"),
        py::arg("taps_y"), py::arg("y_ptr"), py::arg("uv_ptr"), py::arg("out_pitch"), py::arg("coded_w"),
        py::arg("coded_h"), py::arg("stream") = 0, py::arg("mfma") = false, py::arg("strip") = false);
    m.def(
        "composite",
        [](uintptr_t tile, int tile_pitch, int tw, int th, uintptr_t dst, int dst_pitch, int dx, int dy,
           uintptr_t stream) {
            pix::launch_composite(as_ptr<const uint8_t>(tile), tile_pitch, tw, th, as_ptr<uint8_t>(dst), dst_pitch, dx,
                                  dy, as_stream(stream));
            HIP_CHECK(hipGetLastError());
        },
        py::arg("tile_ptr"), py::arg("tile_pitch"), py::arg("tile_w"), py::arg("tile_h"), py::arg("dst_ptr"),
        py::arg("dst_pitch"), py::arg("dx"), py::arg("dy"), py::arg("stream") = 0);
    m.def("lanczos_table", [](int in_size, int out_size) {
        std::vector<int> s;
        std::vector<float> w;
        int taps;
        make_lanczos_table(in_size, out_size, s, w, taps);
        py::array_t<int32_t> sa((py::ssize_t)s.size());
        std::memcpy(sa.mutable_data(), s.data(), s.size() * 4);
        py::array_t<float> wa({(py::ssize_t)out_size, (py::ssize_t)taps});
        std::memcpy(wa.mutable_data(), w.data(), w.size() * 4);
        return py::make_tuple(sa, wa, taps);
    });
    m.attr("BARCODE_CELL") = pix::kBarCell;
    m.attr("BARCODE_X") = pix::kBarX;
    m.attr("BARCODE_Y") = pix::kBarY;

    // ---------------------------------------------------------------- session
    py::class_<SessionConfig>(m, "SessionConfig")
        .def(py::init<>())
        .def_readwrite("width", &SessionConfig::width)
        .def_readwrite("height", &SessionConfig::height)
        .def_readwrite("out_width", &SessionConfig::out_width)
        .def_readwrite("out_height", &SessionConfig::out_height)
        .def_readwrite("fps", &SessionConfig::fps)
        .def_readwrite("noise", &SessionConfig::noise)
        .def_readwrite("content", &SessionConfig::content)
        .def_readwrite("pool_slots", &SessionConfig::pool_slots)
        .def_readwrite("use_graph", &SessionConfig::use_graph)
        .def_readwrite("fake_clock", &SessionConfig::fake_clock)
        .def_readwrite("codec", &SessionConfig::codec)
        .def_readwrite("mask_x0", &SessionConfig::mask_x0)
        .def_readwrite("mask_y0", &SessionConfig::mask_y0)
        .def_readwrite("mask_x1", &SessionConfig::mask_x1)
        .def_readwrite("mask_y1", &SessionConfig::mask_y1)
        .def_readwrite("scale_valu", &SessionConfig::scale_valu)
        .def_readwrite("capture_stream", &SessionConfig::capture_stream)
        .def_readwrite("enc", &SessionConfig::enc);

    py::class_<FrameResult>(m, "FrameResult")
        .def_readonly("frame_id", &FrameResult::frame_id)
        .def_readonly("t_capture_us", &FrameResult::t_capture_us)
        .def_readonly("t_encoded_us", &FrameResult::t_encoded_us)
        .def_readonly("gpu_ms", &FrameResult::gpu_ms)
        .def_readonly("idr", &FrameResult::idr)
        .def_readonly("qp", &FrameResult::qp)
        .def_readonly("psnr_y", &FrameResult::psnr_y)
        .def_readonly("psnr_u", &FrameResult::psnr_u)
        .def_readonly("psnr_v", &FrameResult::psnr_v)
        .def_readonly("psnr_y_masked", &FrameResult::psnr_y_masked)
        .def_readonly("deblocked", &FrameResult::deblocked)
        .def_readonly("db_coherent", &FrameResult::db_coherent)
        .def_readonly("db_moving", &FrameResult::db_moving)
        .def_property_readonly("au", [](const FrameResult& r) { return to_bytes(r.au); });

    m.def(
        "run_sessions",
        [](std::vector<Session*> ss, int n_frames, int depth) {
            py::gil_scoped_release rel;
            return run_sessions(ss, n_frames, depth);
        },
        py::arg("sessions"), py::arg("n_frames"), py::arg("depth") = 2,
        "K sessions driven concurrently, one host thread each; returns [[FrameResult]] per session");
    py::class_<PacedStats>(m, "PacedStats")
        .def_readonly("slots", &PacedStats::slots)
        .def_readonly("late_slots", &PacedStats::late_slots)
        .def_readonly("lat_ms", &PacedStats::lat_ms)
        .def_readonly("idr_late", &PacedStats::idr_late)
        .def_readonly("idr_lat_ms", &PacedStats::idr_lat_ms);
    m.def(
        "run_sessions_paced",
        [](std::vector<Session*> ss, int fps, double seconds, int threads, int idr_slot) {
            py::gil_scoped_release rel;
            return run_sessions_paced(ss, fps, seconds, threads, idr_slot);
        },
        py::arg("sessions"), py::arg("fps"), py::arg("seconds"), py::arg("threads") = 8, py::arg("idr_slot") = -1,
        "K sessions paced at fps for `seconds` by `threads` host threads (one frame in flight each); "
        "idr_slot >= 0: every session codes a forced IDR in that slot");
    py::class_<Session>(m, "Session")
        .def(py::init<const SessionConfig&>())
        .def(
            "step",
            [](Session& s, bool force_idr) {
                py::gil_scoped_release rel;
                return s.step(force_idr);
            },
            py::arg("force_idr") = false)
        .def(
            "submit",
            [](Session& s, bool force_idr) {
                py::gil_scoped_release rel;
                s.submit_synthetic(force_idr);
            },
            py::arg("force_idr") = false)
        .def(
            "submit_bgrx",
            [](Session& s, py::array_t<uint8_t, py::array::c_style> img, bool force_idr) {
                if (img.ndim() != 3 || img.shape(2) != 4) throw std::invalid_argument("expect HxWx4 BGRx");
                if (img.shape(0) != s.config().height || img.shape(1) != s.config().width)
                    throw std::invalid_argument("frame size != session desktop size");
                const uint8_t* p = img.data();
                const int pitch = (int)img.shape(1) * 4;
                py::gil_scoped_release rel;
                s.submit_bgrx(p, pitch, force_idr);
            },
            py::arg("frame"), py::arg("force_idr") = false)
        .def("register_host_buffer",
             [](Session& s, uintptr_t addr, size_t bytes) { s.register_host_buffer(as_ptr<const void>(addr), bytes); },
             py::arg("addr"), py::arg("nbytes"))
        .def(
            "submit_bgrx_ptr",
            [](Session& s, uintptr_t addr, int pitch, size_t nbytes, bool force_idr) {
                py::gil_scoped_release rel;
                s.submit_bgrx_span(as_ptr<const uint8_t>(addr), pitch, nbytes, force_idr);
            },
            py::arg("addr"), py::arg("pitch"), py::arg("nbytes"), py::arg("force_idr") = false,
            "BGRx frame at a host address with `nbytes` readable (zero-copy inside a registered buffer; "
            "ValueError if the frame does not fit)")
        .def(
            "submit_bgrx_damage",
            [](Session& s, uintptr_t addr, int pitch, size_t nbytes, std::vector<std::pair<int, int>> bands,
               bool force_idr) {
                py::gil_scoped_release rel;
                s.submit_bgrx_damage(as_ptr<const uint8_t>(addr), pitch, nbytes, bands, force_idr);
            },
            py::arg("addr"), py::arg("pitch"), py::arg("nbytes"), py::arg("bands"), py::arg("force_idr") = false,
            "damage-driven capture: DMA only the changed row bands [(y0, y1), ...] into the session's "
            "device-resident screen (the first call uploads everything); ValueError for a band outside the frame")
        .def("invalidate_screen", &Session::invalidate_screen,
             "the next submit_bgrx_damage uploads the whole frame (e.g. after the capture lost damage events)")
        .def_property_readonly("damage_bytes_uploaded", &Session::damage_bytes_uploaded)
        .def("collect",
             [](Session& s) {
                 py::gil_scoped_release rel;
                 return s.collect();
             })
        .def("set_cursor", &Session::set_cursor)
        .def("request_idr", &Session::request_idr)
        .def("set_bitrate", &Session::set_bitrate)
        .def_property_readonly("stream", [](Session& s) { return reinterpret_cast<uintptr_t>(s.stream()); })
        .def_property_readonly("capture_stream_active", &Session::capture_stream_active)
        .def_property_readonly("nv12_y_ptr", [](Session& s) { return reinterpret_cast<uintptr_t>(s.nv12_y()); })
        .def_property_readonly("nv12_uv_ptr", [](Session& s) { return reinterpret_cast<uintptr_t>(s.nv12_uv()); })
        .def_property_readonly("nv12_pitch", &Session::nv12_pitch)
        .def_property_readonly("graphs_built", &Session::graphs_built)
        .def_property_readonly("in_flight", &Session::in_flight)
        .def_property_readonly("depth", &Session::depth)
        .def_property_readonly("codec", [](Session& s) { return std::string(s.encoder().codec()); })
        .def("nv12",
             [](Session& s) {
                 const auto& g = s.encoder().geometry();
                 return py::make_tuple(copy_plane(s.nv12_y(), g.pitch, g.coded_w, g.coded_h),
                                       copy_plane(s.nv12_uv(), g.pitch, g.coded_w, g.coded_h / 2));
             })
        .def("recon",
             [](Session& s) {
                 const auto& g = s.encoder().geometry();
                 return py::make_tuple(copy_plane(s.encoder().recon_y(), g.pitch, g.coded_w, g.coded_h),
                                       copy_plane(s.encoder().recon_uv(), g.pitch, g.coded_w, g.coded_h / 2));
             })
        .def_property_readonly("stats", [](Session& s) { return s.encoder().last_stats(); })
        .def("slice_timing",
             [](Session& s) {
                 // HEVC only: per-substream CABAC timing of the last collected picture (GpuHevcEncoder)
                 auto* e = dynamic_cast<hevc::GpuHevcEncoder*>(&s.encoder());
                 if (!e) throw std::invalid_argument("slice_timing: HEVC sessions only");
                 return e->slice_timing();
             })
        .def("cu_token_table", [](Session& s) {
            auto* e = dynamic_cast<hevc::GpuHevcEncoder*>(&s.encoder());
            if (!e) throw std::invalid_argument("cu_token_table: HEVC sessions only");
            return e->cu_token_table();
        });
}
