// RTP payloader for VP8 (RFC 7741) -- the transport of WEBRTC_ENCODER=vp8enc (reference
// README.md:21,35; the reference's GStreamer pipeline uses rtpvp8pay).  Every packet carries the
// payload descriptor with the extension byte and a 15-bit PictureID (X = I = M = 1); the first
// packet of a frame has S = 1, PID = 0 (frames are split at the MTU budget, not at partition
// boundaries, which RFC 7741 section 4.4 permits); the marker bit ends the frame.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

class RtpVp8Packetizer {
   public:
    RtpVp8Packetizer(uint32_t ssrc, uint8_t payload_type, size_t max_payload = 1150, uint16_t first_seq = 0,
                     uint16_t first_picture_id = 0);
    // Packetize one VP8 frame with the given 90 kHz timestamp.
    std::vector<std::string> packetize(const std::string& frame, uint32_t timestamp);
    uint16_t next_seq() const { return seq_; }
    uint16_t next_picture_id() const { return pic_; }
    uint32_t ssrc() const { return ssrc_; }
    uint64_t packets() const { return packets_; }
    uint64_t octets() const { return octets_; }

   private:
    uint32_t ssrc_;
    uint8_t pt_;
    size_t max_payload_;
    uint16_t seq_;
    uint16_t pic_;  // 15 bits
    uint64_t packets_ = 0, octets_ = 0;
};

}  // namespace net
}  // namespace mx
