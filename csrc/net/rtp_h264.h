// RTP payloader for H.264 (RFC 6184, packetization-mode=1): single NAL unit packets,
// STAP-A aggregation of small NAL units (SPS+PPS), FU-A fragmentation above the MTU budget.
// Replaces GStreamer `rtph264pay` in the reference's selkies pipeline.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

// Split an Annex-B byte stream into NAL units (without start codes).
std::vector<std::string> split_annexb(const std::string& au);

class RtpH264Packetizer {
   public:
    RtpH264Packetizer(uint32_t ssrc, uint8_t payload_type, size_t max_payload = 1150, uint16_t first_seq = 0);
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
