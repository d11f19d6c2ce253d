// pybind11 bindings of the native RFB encoder (ZRLE) and host tile diff.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../rfb/zrle.h"

namespace py = pybind11;
using namespace mx::rfb;

namespace {
using Frame = py::array_t<uint8_t, py::array::c_style>;
void check_frame(const Frame& f) {
    if (f.ndim() != 3 || f.shape(2) != 4) throw std::invalid_argument("frame must be (H, W, 4) uint8 BGRx");
}
}  // namespace

void register_rfb(py::module& m) {
    py::module r = m.def_submodule("rfb", "RFB/VNC encoders: ZRLE, tile diff");
    py::class_<ZrleEncoder>(r, "ZrleEncoder")
        .def(py::init<int>(), py::arg("level") = 6)
        .def(
            "encode",
            [](ZrleEncoder& z, Frame f, int x, int y, int w, int h, std::vector<int> perm) {
                check_frame(f);
                if (perm.size() != 3) throw std::invalid_argument("perm needs 3 entries");
                if (x < 0 || y < 0 || w <= 0 || h <= 0 || x + w > f.shape(1) || y + h > f.shape(0))
                    throw std::invalid_argument("rectangle outside the frame");
                std::string out;
                {
                    py::gil_scoped_release rel;
                    out = z.encode(f.data(), (size_t)f.shape(1) * 4, x, y, w, h, perm.data());
                }
                return py::bytes(out);
            },
            py::arg("frame"), py::arg("x"), py::arg("y"), py::arg("w"), py::arg("h"), py::arg("perm"))
        .def_property_readonly("stats", &ZrleEncoder::stats);
    r.def(
        "tile_diff",
        [](Frame cur, Frame prev, int tile) {
            check_frame(cur);
            check_frame(prev);
            if (cur.shape(0) != prev.shape(0) || cur.shape(1) != prev.shape(1)) throw std::invalid_argument("shape");
            const int h = (int)cur.shape(0), w = (int)cur.shape(1);
            std::vector<uint8_t> fl;
            {
                py::gil_scoped_release rel;
                fl = tile_diff(cur.data(), prev.data(), (size_t)w * 4, w, h, tile);
            }
            const int tw = (w + tile - 1) / tile, th = (h + tile - 1) / tile;
            py::array_t<uint8_t> a({th, tw});
            std::memcpy(a.mutable_data(), fl.data(), fl.size());
            return a;
        },
        py::arg("cur"), py::arg("prev"), py::arg("tile") = 64);
}
