#include "rtp_vp8.h"

#include <algorithm>
#include <stdexcept>

namespace mx {
namespace net {

namespace {
constexpr size_t kDescriptor = 4;  // X|R|N|S|R|PID, I|L|T|K|RSV, M|PictureID (15 bits)
}

RtpVp8Packetizer::RtpVp8Packetizer(uint32_t ssrc, uint8_t pt, size_t max_payload, uint16_t first_seq,
                                   uint16_t first_picture_id)
    : ssrc_(ssrc), pt_(pt), max_payload_(max_payload), seq_(first_seq), pic_(first_picture_id & 0x7fff) {
    if (max_payload < 64) throw std::invalid_argument("RTP payload budget too small");
}

std::vector<std::string> RtpVp8Packetizer::packetize(const std::string& frame, uint32_t ts) {
    std::vector<std::string> out;
    if (frame.empty()) return out;
    // N (non-reference) stays 0: every frame this encoder emits updates the last-frame buffer
    const size_t chunk = max_payload_ - kDescriptor;
    const size_t n = (frame.size() + chunk - 1) / chunk;
    out.reserve(n);
    for (size_t k = 0, off = 0; k < n; ++k) {
        const size_t len = std::min(chunk, frame.size() - off);
        std::string p(12 + kDescriptor, '\0');
        p[0] = (char)0x80;
        p[1] = (char)((k + 1 == n ? 0x80 : 0) | (pt_ & 0x7f));
        p[2] = (char)(seq_ >> 8);
        p[3] = (char)seq_;
        for (int i = 0; i < 4; ++i) p[4 + i] = (char)(ts >> (24 - 8 * i));
        for (int i = 0; i < 4; ++i) p[8 + i] = (char)(ssrc_ >> (24 - 8 * i));
        p[12] = (char)(0x80 | (k == 0 ? 0x10 : 0));  // X, S on the frame's first packet, PID 0
        p[13] = (char)0x80;                            // I: PictureID present
        p[14] = (char)(0x80 | (pic_ >> 8));            // M: 15-bit PictureID
        p[15] = (char)pic_;
        p.append(frame, off, len);
        octets_ += kDescriptor + len;
        ++packets_;
        ++seq_;
        off += len;
        out.push_back(std::move(p));
    }
    pic_ = (uint16_t)((pic_ + 1) & 0x7fff);
    return out;
}

}  // namespace net
}  // namespace mx
