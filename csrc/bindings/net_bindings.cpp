// pybind11 bindings of the native transport pieces (SRTP, DTLS-SRTP, RTP H.264).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../net/dtls.h"
#include "../net/rtp_h264.h"
#include "../net/rtp_h265.h"
#include "../net/srtp.h"

namespace py = pybind11;
using namespace mx::net;

namespace {
py::bytes B(const std::string& s) { return py::bytes(s); }
std::vector<py::bytes> BV(const std::vector<std::string>& v) {
    std::vector<py::bytes> o;
    o.reserve(v.size());
    for (const auto& s : v) o.emplace_back(s);
    return o;
}
}  // namespace

void register_net(py::module& m) {
    py::module n = m.def_submodule("net", "WebRTC transport: SRTP, DTLS-SRTP, RTP/H.264");
    py::class_<SrtpSession>(n, "SrtpSession")
        .def(py::init<const std::string&, const std::string&>(), py::arg("master_key"), py::arg("master_salt"))
        .def("protect_rtp", [](SrtpSession& s, py::bytes p) { return B(s.protect_rtp(p)); })
        .def("unprotect_rtp", [](SrtpSession& s, py::bytes p) { return B(s.unprotect_rtp(p)); })
        .def("protect_rtcp", [](SrtpSession& s, py::bytes p) { return B(s.protect_rtcp(p)); })
        .def("unprotect_rtcp", [](SrtpSession& s, py::bytes p) { return B(s.unprotect_rtcp(p)); })
        .def_property_readonly("rtp_key", [](SrtpSession& s) { return B(s.rtp_key()); })
        .def_property_readonly("rtp_salt", [](SrtpSession& s) { return B(s.rtp_salt()); })
        .def_property_readonly("rtp_auth", [](SrtpSession& s) { return B(s.rtp_auth()); })
        .def_property_readonly("rtcp_key", [](SrtpSession& s) { return B(s.rtcp_key()); })
        .def_static("aes_cm_keystream", [](py::bytes k, py::bytes iv, size_t n) {
            return B(SrtpSession::aes_cm_keystream(k, iv, n));
        });
    py::class_<DtlsEndpoint>(n, "DtlsEndpoint")
        .def(py::init<bool, int>(), py::arg("server"), py::arg("mtu") = 1200)
        .def_property_readonly("fingerprint", &DtlsEndpoint::fingerprint)
        .def("start", [](DtlsEndpoint& d) { return BV(d.start()); })
        .def("feed", [](DtlsEndpoint& d, py::bytes b) { return BV(d.feed(b)); })
        .def("tick", [](DtlsEndpoint& d) { return BV(d.tick()); })
        .def_property_readonly("handshake_done", &DtlsEndpoint::handshake_done)
        .def_property_readonly("failed", &DtlsEndpoint::failed)
        .def_property_readonly("error", &DtlsEndpoint::error)
        .def_property_readonly("peer_fingerprint", &DtlsEndpoint::peer_fingerprint)
        .def_property_readonly("srtp_profile", &DtlsEndpoint::srtp_profile)
        .def("export_srtp_keys", [](DtlsEndpoint& d) { return B(d.export_srtp_keys()); });
    py::class_<RtpH264Packetizer>(n, "RtpH264Packetizer")
        .def(py::init<uint32_t, uint8_t, size_t, uint16_t>(), py::arg("ssrc"), py::arg("payload_type"),
             py::arg("max_payload") = 1150, py::arg("first_seq") = 0)
        .def("packetize", [](RtpH264Packetizer& p, py::bytes au, uint32_t ts) { return BV(p.packetize(au, ts)); })
        .def_property_readonly("next_seq", &RtpH264Packetizer::next_seq)
        .def_property_readonly("ssrc", &RtpH264Packetizer::ssrc)
        .def_property_readonly("packets", &RtpH264Packetizer::packets)
        .def_property_readonly("octets", &RtpH264Packetizer::octets);
    py::class_<RtpH265Packetizer>(n, "RtpH265Packetizer")
        .def(py::init<uint32_t, uint8_t, size_t, uint16_t>(), py::arg("ssrc"), py::arg("payload_type"),
             py::arg("max_payload") = 1150, py::arg("first_seq") = 0)
        .def("packetize", [](RtpH265Packetizer& p, py::bytes au, uint32_t ts) { return BV(p.packetize(au, ts)); })
        .def_property_readonly("next_seq", &RtpH265Packetizer::next_seq)
        .def_property_readonly("ssrc", &RtpH265Packetizer::ssrc)
        .def_property_readonly("packets", &RtpH265Packetizer::packets)
        .def_property_readonly("octets", &RtpH265Packetizer::octets);
    n.def("split_annexb", [](py::bytes au) { return BV(split_annexb(au)); });
}
