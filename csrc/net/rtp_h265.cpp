#include "rtp_h265.h"

#include <algorithm>
#include <stdexcept>

#include "rtp_h264.h"  // split_annexb

namespace mx {
namespace net {

RtpH265Packetizer::RtpH265Packetizer(uint32_t ssrc, uint8_t pt, size_t max_payload, uint16_t first_seq)
    : ssrc_(ssrc), pt_(pt), max_payload_(max_payload), seq_(first_seq) {
    if (max_payload < 64) throw std::invalid_argument("RTP payload budget too small");
}

std::string RtpH265Packetizer::header(bool marker, uint32_t ts) {
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

std::vector<std::string> RtpH265Packetizer::packetize(const std::string& au, uint32_t ts) {
    std::vector<std::string> nals = split_annexb(au);
    nals.erase(std::remove_if(nals.begin(), nals.end(), [](const std::string& n) { return n.size() < 3; }), nals.end());
    std::vector<std::string> payloads;
    size_t i = 0;
    while (i < nals.size()) {
        // AP: consecutive small NAL units; PayloadHdr F = OR, LayerId / TID = minimum
        size_t j = i, total = 2;
        while (j < nals.size() && total + 2 + nals[j].size() <= max_payload_ && nals[j].size() < 512) {
            total += 2 + nals[j].size();
            ++j;
        }
        if (j - i >= 2) {
            uint8_t f = 0, layer = 63, tid = 7;
            for (size_t k = i; k < j; ++k) {
                const uint8_t h0 = (uint8_t)nals[k][0], h1 = (uint8_t)nals[k][1];
                f |= h0 & 0x80;
                layer = std::min<uint8_t>(layer, (uint8_t)(((h0 & 1) << 5) | (h1 >> 3)));
                tid = std::min<uint8_t>(tid, h1 & 7);
            }
            std::string p;
            p.push_back((char)(f | (48 << 1) | (layer >> 5)));
            p.push_back((char)(((layer & 31) << 3) | tid));
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
        } else {  // FU: PayloadHdr (type 49) + FU header (S, E, FuType) + fragment
            const uint8_t h0 = (uint8_t)nal[0], h1 = (uint8_t)nal[1];
            const uint8_t type = (h0 >> 1) & 63;
            size_t off = 2;
            const size_t chunk = max_payload_ - 3;
            while (off < nal.size()) {
                const size_t len = std::min(chunk, nal.size() - off);
                uint8_t fu = type;
                if (off == 2) fu |= 0x80;
                if (off + len == nal.size()) fu |= 0x40;
                std::string p;
                p.reserve(len + 3);
                p.push_back((char)((h0 & 0x81) | (49 << 1)));
                p.push_back((char)h1);
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
