// pybind11 bindings of the audio helpers (G.711 mu-law, decimator).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "../audio/audio.h"

namespace py = pybind11;
using namespace mx::audio;

void register_audio(py::module& m) {
    py::module a = m.def_submodule("audio", "desktop audio: G.711 mu-law, decimation");
    a.def("encode_ulaw", [](py::array_t<int16_t, py::array::c_style> pcm) {
        return py::bytes(encode_ulaw(pcm.data(), (size_t)pcm.size()));
    });
    a.def("decode_ulaw", [](py::bytes b) {
        const std::string s = b;
        py::array_t<int16_t> out((py::ssize_t)s.size());
        for (size_t i = 0; i < s.size(); ++i) out.mutable_data()[i] = ulaw_to_linear((uint8_t)s[i]);
        return out;
    });
    py::class_<Decimator>(a, "Decimator")
        .def(py::init<int, int, int>(), py::arg("factor"), py::arg("channels"), py::arg("taps_per_phase") = 16)
        .def("process",
             [](Decimator& d, py::array_t<int16_t, py::array::c_style> x) {
                 if (x.size() % d.channels()) throw std::invalid_argument("sample count not a multiple of channels");
                 const auto out = d.process(x.data(), (size_t)x.size() / d.channels());
                 py::array_t<int16_t> r((py::ssize_t)out.size());
                 std::copy(out.begin(), out.end(), r.mutable_data());
                 return r;
             })
        .def_property_readonly("factor", &Decimator::factor);
}
