// RTP payloader for HEVC (RFC 7798, no DONL): single NAL unit packets, aggregation packets
// (AP, type 48) for small NAL units such as VPS+SPS+PPS, fragmentation units (FU, type 49)
// above the MTU budget.  The H.265 counterpart of rtp_h264.h for WEBRTC_ENCODER=mxh265enc.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

class RtpH265Packetizer {
   public:
    RtpH265Packetizer(uint32_t ssrc, uint8_t payload_type, size_t max_payload = 1150, uint16_t first_seq = 0);
    // Packetize one access unit with the given 90 kHz timestamp; marker on the last packet.
    std::vector<std::string> packetize(const std::string& annexb_au, uint32_t timestamp);
    uint16_t next_seq() const { return seq_; }
    uint32_t ssrc() const { return ssrc_; }
    uint64_t packets() const { return packets_; }
    uint64_t octets() const { return octets_; }

   private:
    std::string header(bool marker, uint32_t ts);
    uint32_t ssrc_;
    uint8_t pt_;
    size_t max_payload_;
    uint16_t seq_;
    uint64_t packets_ = 0, octets_ = 0;
};

}  // namespace net
}  // namespace mx
