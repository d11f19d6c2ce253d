// Host-side ASan/UBSan driver for the native code that parses or produces untrusted /
// variable-length data: CPU H.264 / HEVC / VP8 encoders (same MB cores as the
// HIP kernels), SRTP/SRTCP, DTLS-SRTP handshake, RTP H.264 / H.265 / VP8 packetizers, Annex-B
// splitter.
// Built by tools/sanitize.sh with -fsanitize on the host side only; no GPU is touched.
#include <arpa/inet.h>
#include <cstdio>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../csrc/codec/h264_encoder.h"
#include "../csrc/codec/hevc_encoder.h"
#include "../csrc/codec/vp8_encoder.h"
#include "../csrc/net/dtls.h"
#include "../csrc/net/rtp_h264.h"
#include "../csrc/net/rtp_h265.h"
#include "../csrc/net/rtp_sender.h"
#include "../csrc/net/rtp_vp8.h"
#include "../csrc/net/sctp.h"
#include "../csrc/net/srtp.h"

using namespace mx;

static int fails = 0;
#define CHECK(c)                                                  \
    do {                                                          \
        if (!(c)) {                                               \
            std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            ++fails;                                              \
        }                                                         \
    } while (0)

static void encoder_pass(std::mt19937& rng) {
    const int sizes[][2] = {{176, 144}, {100, 60}, {64, 48}};
    for (auto& s : sizes) {
        for (int subpel = 0; subpel < 2; ++subpel) {
            h264::EncoderConfig c;
            c.width = s[0];
            c.height = s[1];
            c.bitrate_kbps = 0;
            c.qp = 10 + (int)(rng() % 36);
            c.subpel = subpel;
            c.search_range = 8;
            h264::CpuH264Encoder enc(c);
            const int cw = enc.coded_pitch(), ch = (s[1] + 15) / 16 * 16;
            std::vector<uint8_t> y((size_t)cw * ch), uv((size_t)cw * ch / 2);
            for (int f = 0; f < 4; ++f) {
                for (int r = 0; r < ch; ++r)
                    for (int x = 0; x < cw; ++x)
                        y[(size_t)r * cw + x] = (uint8_t)((x * 3 + r * 2 + f * 5) ^ ((f & 1) ? (rng() & 31) : 0));
                for (auto& v : uv) v = (uint8_t)(128 + (int)(rng() % 32) - 16);
                const auto& au = enc.encode(y.data(), uv.data(), cw, f == 0);
                CHECK(au.size() > 4);
                CHECK(au[0] == 0 && au[1] == 0);
            }
        }
    }
}

static void hevc_pass(std::mt19937& rng) {
    const int sizes[][3] = {{176, 144, 60}, {100, 60, 60}, {352, 288, 30}};  // 352x288@30: two-row slices
    for (auto& s : sizes) {
        h264::EncoderConfig c;
        c.width = s[0];
        c.height = s[1];
        c.fps = s[2];
        c.bitrate_kbps = 0;
        c.qp = 4 + (int)(rng() % 46);
        c.search_range = 8;
        hevc::CpuHevcEncoder enc(c);
        const int cw = enc.coded_pitch(), ch = (s[1] + 15) / 16 * 16;
        std::vector<uint8_t> y((size_t)cw * ch), uv((size_t)cw * ch / 2);
        for (int f = 0; f < 4; ++f) {
            for (int r = 0; r < ch; ++r)
                for (int x = 0; x < cw; ++x)
                    y[(size_t)r * cw + x] = (uint8_t)((x * 3 + r * 2 + f * 5) ^ ((r > ch / 2) ? (rng() & 255) : 0));
            for (auto& v : uv) v = (uint8_t)(128 + (int)(rng() % 32) - 16);
            const auto& au = enc.encode(y.data(), uv.data(), cw, f == 0);
            CHECK(au.size() > 6);
            CHECK(au[0] == 0 && au[1] == 0 && au[2] == 0 && au[3] == 1);
        }
    }
}

static void vp8_pass(std::mt19937& rng) {
    const int sizes[][2] = {{176, 144}, {100, 60}, {64, 48}, {320, 192}};
    for (auto& s : sizes) {
        h264::EncoderConfig c;
        c.width = s[0];
        c.height = s[1];
        c.bitrate_kbps = (rng() & 1) ? 0 : 300;
        c.qp = 4 + (int)(rng() % 46);
        c.search_range = 8;
        vp8::CpuVp8Encoder enc(c);
        const int cw = enc.coded_pitch(), ch = (s[1] + 15) / 16 * 16;
        std::vector<uint8_t> y((size_t)cw * ch), uv((size_t)cw * ch / 2);
        for (int f = 0; f < 5; ++f) {
            for (int r = 0; r < ch; ++r)
                for (int x = 0; x < cw; ++x)
                    y[(size_t)r * cw + x] = (uint8_t)(((x + 3 * f) * 3 + r * 2) ^ ((r > ch / 2) ? (rng() & 255) : 0));
            for (auto& v : uv) v = (uint8_t)(128 + (int)(rng() % 64) - 32);
            const auto& fr = enc.encode(y.data(), uv.data(), cw, f == 3);
            CHECK(fr.size() > 3);
            CHECK(((fr[0] & 1) == 0) == (f == 0 || f == 3));  // frame tag: key frames
        }
    }
}

static std::string rnd(std::mt19937& rng, size_t n) {
    std::string s(n, '\0');
    for (auto& ch : s) ch = (char)(rng() & 0xff);
    return s;
}

static void srtp_pass(std::mt19937& rng) {
    const std::string k = rnd(rng, 16), salt = rnd(rng, 14);
    net::SrtpSession tx(k, salt), rx(k, salt);
    for (int i = 0; i < 300; ++i) {
        std::string pkt = rnd(rng, 12 + rng() % 1200);
        pkt[0] = (char)0x80;
        pkt[2] = (char)(i >> 8);
        pkt[3] = (char)i;
        const std::string p = tx.protect_rtp(pkt);
        CHECK(rx.unprotect_rtp(p) == pkt);
        std::string bad = p;
        bad[bad.size() / 2] ^= 1;
        CHECK(rx.unprotect_rtp(bad).empty());
        CHECK(rx.unprotect_rtp(p.substr(0, rng() % 22)).empty());
    }
    for (int i = 0; i < 50; ++i) {
        std::string r = rnd(rng, 8 + rng() % 100);
        r[0] = (char)0x81;
        r[1] = (char)206;
        CHECK(rx.unprotect_rtcp(tx.protect_rtcp(r)) == r);
    }
}

static void rtp_pass(std::mt19937& rng) {
    for (int i = 0; i < 200; ++i) {
        std::string au = rnd(rng, rng() % 6000);
        if (i % 2) au = std::string("\x00\x00\x00\x01\x67", 5) + au + std::string("\x00\x00\x01\x65", 4) + au;
        net::RtpH264Packetizer pk((uint32_t)rng(), 96, 64 + rng() % 1200, (uint16_t)rng());
        for (const auto& p : pk.packetize(au, (uint32_t)rng())) CHECK(p.size() >= 12);
        net::RtpH265Packetizer pk5((uint32_t)rng(), 97, 64 + rng() % 1200, (uint16_t)rng());
        for (const auto& p : pk5.packetize(au, (uint32_t)rng())) CHECK(p.size() >= 12);
        net::RtpVp8Packetizer pk8((uint32_t)rng(), 98, 64 + rng() % 1200, (uint16_t)rng(), (uint16_t)rng());
        for (const auto& p : pk8.packetize(au, (uint32_t)rng())) CHECK(p.size() > 16);
        (void)net::split_annexb(au);
    }
}

static void dtls_pass() {
    net::DtlsEndpoint srv(true), cli(false);
    auto to_srv = cli.start();
    for (int round = 0; round < 20 && !(srv.handshake_done() && cli.handshake_done()); ++round) {
        std::vector<std::string> to_cli;
        for (const auto& d : to_srv)
            for (auto& o : srv.feed(d)) to_cli.push_back(o);
        to_srv.clear();
        for (const auto& d : to_cli)
            for (auto& o : cli.feed(d)) to_srv.push_back(o);
    }
    CHECK(srv.handshake_done() && cli.handshake_done());
    CHECK(srv.export_srtp_keys() == cli.export_srtp_keys());
    for (const auto& d : cli.write(std::string(1100, 'x'))) (void)srv.feed(d);
    auto app = srv.take_app_data();
    CHECK(app.size() == 1 && app[0].size() == 1100);
    net::DtlsEndpoint junk(true);
    std::mt19937 rng(7);
    for (int i = 0; i < 50; ++i) (void)junk.feed(rnd(rng, 1 + rng() % 300));
}

// Two data-channel endpoints over a link that drops 10 % of packets; meanwhile every packet
// is also fed, mutated or truncated, into a third endpoint that must reject it cleanly.
static void sctp_pass(std::mt19937& rng) {
    net::DataChannelEndpoint a(false), b(true), victim(true);
    int64_t t = 0;
    a.sctp().set_clock(0);
    b.sctp().set_clock(0);
    std::vector<std::string> qa = a.connect(), qb;
    int id = -1;
    std::vector<std::string> sent;
    size_t got = 0, n_sent = 0, sent_bytes = 0, got_bytes = 0;
    for (int step = 0; step < 6000; ++step) {
        if (step == 50) {
            auto r = a.open("input");
            id = r.first;
            for (auto& p : r.second) qa.push_back(p);
        }
        if (id >= 0 && step > 60 && step < 400 && step % 4 == 0) {
            std::string m = rnd(rng, 1 + rng() % 9000);
            sent_bytes += m.size();
            ++n_sent;
            for (auto& p : a.send((uint16_t)id, m, true)) qa.push_back(p);
        }
        std::vector<std::string> na, nb;
        for (auto& p : qa) {
            std::string m = p;
            if (!m.empty()) m[rng() % m.size()] ^= (char)(1 + rng() % 255);
            (void)victim.feed(rng() % 2 ? m : m.substr(0, rng() % (m.size() + 1)));
            if (rng() % 10) for (auto& o : b.feed(p)) nb.push_back(o);
        }
        for (auto& p : qb)
            if (rng() % 10) for (auto& o : a.feed(p)) na.push_back(o);
        qa.swap(na);
        qb.swap(nb);
        t += 10;
        a.sctp().set_clock(t);
        b.sctp().set_clock(t);
        for (auto& p : a.tick()) qa.push_back(p);
        for (auto& p : b.tick()) qb.push_back(p);
        for (auto& e : b.take_events())
            if (e.kind == net::DataChannelEvent::Message) ++got, got_bytes += e.data.size();
    }
    CHECK(a.sctp().established() && b.sctp().established());
    CHECK(n_sent > 50 && got == n_sent && got_bytes == sent_bytes);
    CHECK(a.sctp().buffered_amount() == 0);
}

// Two-phase HEVC CABAC (bin tokens) against direct coding on random slices, and the native RTP
// send path (packetize -> NACK history -> SRTP -> sendto) into a local UDP socket.
static void token_and_sender_pass(std::mt19937& rng) {
    CHECK(hevc::token_selftest(rng() & 0xffff, 60) == 60);
    const int rx = socket(AF_INET, SOCK_DGRAM, 0), tx = socket(AF_INET, SOCK_DGRAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    CHECK(bind(rx, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0);
    socklen_t len = sizeof a;
    CHECK(getsockname(rx, reinterpret_cast<sockaddr*>(&a), &len) == 0);
    net::UdpPeer peer(tx, "127.0.0.1", ntohs(a.sin_port));
    net::RtpHistory hist(64);
    net::SrtpSession srtp(std::string(16, 'k'), std::string(14, 's'));
    net::RtpH264Packetizer pk(0x1234, 96, 1150, 100);
    std::string au;
    for (int n = 0; n < 3; ++n) {
        au += std::string("\x00\x00\x00\x01", 4);
        const size_t nal = 100 + rng() % 4000;
        au.push_back((char)0x65);
        for (size_t i = 1; i < nal; ++i) au.push_back((char)(1 + rng() % 255));
    }
    const std::vector<std::string> raw = pk.packetize(au, 9000);
    CHECK(net::send_rtp_packets(raw, srtp, hist, peer) == (int)raw.size());
    for (const std::string& p : raw) {
        const uint16_t seq = (uint16_t)(((uint8_t)p[2] << 8) | (uint8_t)p[3]);
        const std::string* h = hist.get(seq);
        CHECK(h != nullptr && *h == p);
    }
    char buf[2048];
    int got = 0;
    while (got < (int)raw.size() && recv(rx, buf, sizeof buf, MSG_DONTWAIT) > 0) ++got;
    CHECK(got == (int)raw.size());
    close(rx);
    close(tx);
}

int main() {
    std::mt19937 rng(12345);
    token_and_sender_pass(rng);
    encoder_pass(rng);
    hevc_pass(rng);
    vp8_pass(rng);
    srtp_pass(rng);
    rtp_pass(rng);
    dtls_pass();
    sctp_pass(rng);
    std::printf("sanitize: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}
