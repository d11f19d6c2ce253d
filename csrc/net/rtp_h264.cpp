#include "rtp_h264.h"

#include <stdexcept>

namespace mx {
namespace net {

std::vector<std::string> split_annexb(const std::string& au) {
    std::vector<std::string> nals;
    const size_t n = au.size();
    const uint8_t* b = (const uint8_t*)au.data();
    std::vector<size_t> starts;
    for (size_t i = 0; i + 3 <= n; ++i)
        if (b[i] == 0 && b[i + 1] == 0 && b[i + 2] == 1) {
            starts.push_back(i + 3);
            i += 2;
        }
    for (size_t k = 0; k < starts.size(); ++k) {
        size_t e = (k + 1 < starts.size()) ? starts[k + 1] - 3 : n;
        while (e > starts[k] && b[e - 1] == 0) --e;  // 4-byte start codes / trailing zeros
        if (e > starts[k]) nals.emplace_back(au, starts[k], e - starts[k]);
    }
    return nals;
}

RtpH264Packetizer::RtpH264Packetizer(uint32_t ssrc, uint8_t pt, size_t max_payload, uint16_t first_seq)
    : ssrc_(ssrc), pt_(pt), max_payload_(max_payload), seq_(first_seq) {
    if (max_payload < 64) throw std::invalid_argument("RTP payload budget too small");
}

std::string RtpH264Packetizer::header(bool marker, uint32_t ts) {
    std::string h(12, '\0');
    h[0] = (char)0x80;
    h[1] = (char)((marker ? 0x80 : 0) | (pt_ & 0x7f));
    h[2] = (char)(seq_ >> 8);
    h[3] = (char)seq_;
    for (int i = 0; i < 4; ++i) h[4 + i] = (char)(ts >> (24 - 8 * i));
    for (int i = 0; i < 4; ++i) h[8 + i] = (char)(ssrc_ >> (24 - 8 * i));
    ++seq_;
    return h;
}

std::vector<std::string> RtpH264Packetizer::packetize(const std::string& au, uint32_t ts) {
    const std::vector<std::string> nals = split_annexb(au);
    std::vector<std::string> payloads;
    size_t i = 0;
    while (i < nals.size()) {
        // STAP-A: aggregate consecutive small NAL units (e.g. SPS + PPS + small slices)
        size_t j = i, total = 1;
        uint8_t nri = 0;
        while (j < nals.size() && total + 2 + nals[j].size() <= max_payload_ && nals[j].size() < 512) {
            total += 2 + nals[j].size();
            nri = std::max<uint8_t>(nri, (uint8_t)nals[j][0] & 0x60);
            ++j;
        }
        if (j - i >= 2) {
            std::string p(1, (char)(nri | 24));
            for (size_t k = i; k < j; ++k) {
                p.push_back((char)(nals[k].size() >> 8));
                p.push_back((char)nals[k].size());
                p += nals[k];
            }
            payloads.push_back(std::move(p));
            i = j;
            continue;
        }
        const std::string& nal = nals[i];
        if (nal.size() <= max_payload_) {
            payloads.push_back(nal);
        } else {  // FU-A
            const uint8_t hdr = (uint8_t)nal[0];
            const uint8_t ind = (hdr & 0xe0) | 28;
            size_t off = 1;
            const size_t chunk = max_payload_ - 2;
            while (off < nal.size()) {
                const size_t len = std::min(chunk, nal.size() - off);
                uint8_t fu = hdr & 0x1f;
                if (off == 1) fu |= 0x80;
                if (off + len == nal.size()) fu |= 0x40;
                std::string p;
                p.reserve(len + 2);
                p.push_back((char)ind);
                p.push_back((char)fu);
                p.append(nal, off, len);
                payloads.push_back(std::move(p));
                off += len;
            }
        }
        ++i;
    }
    std::vector<std::string> out;
    out.reserve(payloads.size());
    for (size_t k = 0; k < payloads.size(); ++k) {
        std::string pkt = header(k + 1 == payloads.size(), ts);
        pkt += payloads[k];
        octets_ += payloads[k].size();
        ++packets_;
        out.push_back(std::move(pkt));
    }
    return out;
}

}  // namespace net
}  // namespace mx
