// pybind11 bindings of the native transport pieces (SRTP, DTLS-SRTP, RTP H.264).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../net/dtls.h"
#include "../net/rtp_h264.h"
#include "../net/rtp_counter.h"
#include "../net/rtp_h265.h"
#include "../net/rtp_sender.h"
#include "../net/rtp_vp8.h"
#include "../net/sctp.h"
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
    py::class_<RtpHistory>(n, "RtpHistory")
        .def(py::init<size_t>(), py::arg("n") = 1024)
        .def("get", [](const RtpHistory& h, uint16_t seq) -> py::object {
            const std::string* p = h.get(seq);
            return p ? py::object(py::bytes(*p)) : py::object(py::none());
        });
    py::class_<UdpPeer>(n, "UdpPeer")
        .def(py::init<int, const std::string&, int>(), py::arg("fd"), py::arg("host"), py::arg("port"))
        .def_property_readonly("fd", &UdpPeer::fd);
    // packetize + history + SRTP + sendto of one access unit, GIL released
    auto send_au = [](auto& pk, SrtpSession& srtp, RtpHistory& hist, const UdpPeer& peer, py::bytes au,
                      uint32_t ts) {
        std::string a = au;
        py::gil_scoped_release rel;
        return send_rtp_packets(pk.packetize(a, ts), srtp, hist, peer);
    };
    n.def("send_au", [send_au](RtpH264Packetizer& p, SrtpSession& s, RtpHistory& h, const UdpPeer& u, py::bytes au,
                               uint32_t ts) { return send_au(p, s, h, u, au, ts); });
    n.def("send_au", [send_au](RtpH265Packetizer& p, SrtpSession& s, RtpHistory& h, const UdpPeer& u, py::bytes au,
                               uint32_t ts) { return send_au(p, s, h, u, au, ts); });
    n.def("send_au", [send_au](RtpVp8Packetizer& p, SrtpSession& s, RtpHistory& h, const UdpPeer& u, py::bytes au,
                               uint32_t ts) { return send_au(p, s, h, u, au, ts); });
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
        .def("export_srtp_keys", [](DtlsEndpoint& d) { return B(d.export_srtp_keys()); })
        .def("write", [](DtlsEndpoint& d, py::bytes b) { return BV(d.write(b)); })
        .def("take_app_data", [](DtlsEndpoint& d) { return BV(d.take_app_data()); });
    n.def("crc32c", [](py::bytes b) {
        std::string s = b;
        return crc32c(s.data(), s.size());
    });
    py::class_<SctpStats>(n, "SctpStats")
        .def_readonly("packets_in", &SctpStats::packets_in)
        .def_readonly("packets_out", &SctpStats::packets_out)
        .def_readonly("data_in", &SctpStats::data_in)
        .def_readonly("data_out", &SctpStats::data_out)
        .def_readonly("retransmits", &SctpStats::retransmits)
        .def_readonly("fast_retransmits", &SctpStats::fast_retransmits)
        .def_readonly("t3_expiries", &SctpStats::t3_expiries)
        .def_readonly("abandoned", &SctpStats::abandoned)
        .def_readonly("forward_tsn_out", &SctpStats::forward_tsn_out)
        .def_readonly("forward_tsn_in", &SctpStats::forward_tsn_in)
        .def_readonly("sacks_in", &SctpStats::sacks_in)
        .def_readonly("sacks_out", &SctpStats::sacks_out)
        .def_readonly("dup_tsns", &SctpStats::dup_tsns)
        .def_readonly("bad_checksum", &SctpStats::bad_checksum)
        .def_readonly("bad_tag", &SctpStats::bad_tag)
        .def_readonly("messages_in", &SctpStats::messages_in)
        .def_readonly("messages_out", &SctpStats::messages_out);
    py::class_<SctpAssociation>(n, "SctpAssociation")
        .def(py::init<uint16_t, uint16_t, size_t>(), py::arg("local_port") = 5000, py::arg("remote_port") = 5000,
             py::arg("max_message") = 256 * 1024)
        .def("connect", [](SctpAssociation& a) { return BV(a.connect()); })
        .def("feed", [](SctpAssociation& a, py::bytes p) { return BV(a.feed(p)); })
        .def("send", [](SctpAssociation& a, uint16_t stream, uint32_t ppid, py::bytes d, bool unordered,
                        int max_rtx, int lifetime) { return BV(a.send(stream, ppid, d, unordered, max_rtx, lifetime)); },
             py::arg("stream"), py::arg("ppid"), py::arg("data"), py::arg("unordered") = false,
             py::arg("max_retransmits") = -1, py::arg("lifetime_ms") = -1)
        .def("tick", [](SctpAssociation& a) { return BV(a.tick()); })
        .def("reset_streams", [](SctpAssociation& a, const std::vector<uint16_t>& s) { return BV(a.reset_streams(s)); })
        .def("shutdown", [](SctpAssociation& a) { return BV(a.shutdown()); })
        .def("abort", [](SctpAssociation& a, const std::string& why) { return BV(a.abort(why)); })
        .def("take_messages", [](SctpAssociation& a) {
            py::list out;
            for (auto& m : a.take_messages())
                out.append(py::make_tuple(m.stream, m.ppid, m.unordered, py::bytes(m.data)));
            return out;
        })
        .def("take_reset_streams", &SctpAssociation::take_reset_streams)
        .def_property_readonly("state", [](const SctpAssociation& a) { return (int)a.state(); })
        .def_property_readonly("established", &SctpAssociation::established)
        .def_property_readonly("stats", &SctpAssociation::stats, py::return_value_policy::copy)
        .def_property_readonly("buffered_amount", &SctpAssociation::buffered_amount)
        .def_property_readonly("rto_ms", &SctpAssociation::rto_ms)
        .def_property_readonly("cwnd", &SctpAssociation::cwnd)
        .def_property_readonly("peer_rwnd", &SctpAssociation::peer_rwnd)
        .def_property_readonly("peer_supports_forward_tsn", &SctpAssociation::peer_supports_forward_tsn)
        .def_property_readonly("error", &SctpAssociation::error)
        .def("set_clock", &SctpAssociation::set_clock);
    py::class_<DataChannelEndpoint>(n, "DataChannelEndpoint")
        .def(py::init<bool, uint16_t, uint16_t, size_t>(), py::arg("dtls_server"), py::arg("local_port") = 5000,
             py::arg("remote_port") = 5000, py::arg("max_message") = 256 * 1024)
        .def("connect", [](DataChannelEndpoint& e) { return BV(e.connect()); })
        .def("feed", [](DataChannelEndpoint& e, py::bytes p) { return BV(e.feed(p)); })
        .def("tick", [](DataChannelEndpoint& e) { return BV(e.tick()); })
        .def("open", [](DataChannelEndpoint& e, const std::string& label, const std::string& protocol, bool ordered,
                        int max_rtx, int lifetime) {
                 auto r = e.open(label, protocol, ordered, max_rtx, lifetime);
                 return py::make_tuple(r.first, BV(r.second));
             },
             py::arg("label"), py::arg("protocol") = "", py::arg("ordered") = true, py::arg("max_retransmits") = -1,
             py::arg("max_lifetime_ms") = -1)
        .def("send", [](DataChannelEndpoint& e, uint16_t id, py::bytes d, bool binary) { return BV(e.send(id, d, binary)); },
             py::arg("id"), py::arg("data"), py::arg("binary") = false)
        .def("close", [](DataChannelEndpoint& e, uint16_t id) { return BV(e.close(id)); })
        .def("take_events", [](DataChannelEndpoint& e) {
            py::list out;
            for (auto& ev : e.take_events())
                out.append(py::make_tuple(ev.kind, ev.id, ev.label, ev.protocol, ev.binary, py::bytes(ev.data)));
            return out;
        })
        .def("is_open", &DataChannelEndpoint::is_open)
        .def("label", &DataChannelEndpoint::label)
        .def("channels", &DataChannelEndpoint::channels)
        .def_property_readonly("established", [](DataChannelEndpoint& e) { return e.sctp().established(); })
        .def_property_readonly("stats", [](DataChannelEndpoint& e) { return e.sctp().stats(); })
        .def_property_readonly("buffered_amount", [](DataChannelEndpoint& e) { return e.sctp().buffered_amount(); })
        .def("set_clock", [](DataChannelEndpoint& e, int64_t ms) { e.sctp().set_clock(ms); });
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
    py::class_<RtpVp8Packetizer>(n, "RtpVp8Packetizer")
        .def(py::init<uint32_t, uint8_t, size_t, uint16_t, uint16_t>(), py::arg("ssrc"), py::arg("payload_type"),
             py::arg("max_payload") = 1150, py::arg("first_seq") = 0, py::arg("first_picture_id") = 0)
        .def("packetize", [](RtpVp8Packetizer& p, py::bytes frame, uint32_t ts) { return BV(p.packetize(frame, ts)); })
        .def_property_readonly("next_seq", &RtpVp8Packetizer::next_seq)
        .def_property_readonly("next_picture_id", &RtpVp8Packetizer::next_picture_id)
        .def_property_readonly("ssrc", &RtpVp8Packetizer::ssrc)
        .def_property_readonly("packets", &RtpVp8Packetizer::packets)
        .def_property_readonly("octets", &RtpVp8Packetizer::octets);
    n.def("split_annexb", [](py::bytes au) { return BV(split_annexb(au)); });
    n.def(
        "count_rtp_frames",
        [](int fd, int n_frames, double timeout_s, int64_t ts, int next, bool ok) {
            RtpFrameCount r;
            {
                py::gil_scoped_release rel;
                r = count_rtp_frames(fd, n_frames, timeout_s, RtpLiteState{ts, next, ok});
            }
            py::dict d;
            d["rtp_ts"] = r.rtp_ts;
            d["arrival_us"] = r.arrival_us;
            d["arrival_wall"] = r.arrival_wall;
            d["rtcp"] = BV(r.rtcp);
            d["packets"] = r.packets;
            d["lost"] = r.lost;
            d["datagrams"] = r.datagrams;
            d["timed_out"] = r.timed_out;
            return d;
        },
        py::arg("fd"), py::arg("n_frames"), py::arg("timeout_s"), py::arg("ts") = -1, py::arg("next") = -1,
        py::arg("ok") = true,
        "Count complete RTP frames on a connected UDP socket (recvmmsg, GIL released): rtp_ts, arrival times, "
        "the last RTCP datagrams raw, packets, lost sequence numbers");
}
