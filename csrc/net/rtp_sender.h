// Per-viewer RTP video send path in one native call: packetize an access unit (RFC 6184 / 7798 /
// 7741), keep each raw packet in a sequence-indexed ring for NACK retransmission, SRTP-protect
// and sendto() it on the peer's UDP socket.  The Python send loop used to do this per packet
// (dict insert, protect call, asyncio sendto): ~15 packets per 1080p frame at 8 Mbps, for every
// viewer, on the single event-loop thread that all sessions of a `serve --sessions K` process
// share.  Called with the GIL released.
#pragma once
#include <cstdint>
#include <netinet/in.h>
#include <string>
#include <sys/socket.h>
#include <vector>

#include "srtp.h"

namespace mx {
namespace net {

class RtpHistory {
   public:
    explicit RtpHistory(size_t n = 1024) : slots_(n), seqs_(n, -1) {}
    void put(uint16_t seq, const std::string& raw) {
        slots_[seq % slots_.size()] = raw;
        seqs_[seq % slots_.size()] = seq;
    }
    // raw packet of `seq`, or empty if it has left the ring
    const std::string* get(uint16_t seq) const {
        const size_t i = seq % slots_.size();
        return seqs_[i] == (int)seq ? &slots_[i] : nullptr;
    }

   private:
    std::vector<std::string> slots_;
    std::vector<int> seqs_;
};

class UdpPeer {
   public:
    // fd: the (non-blocking) UDP socket the peer's ICE pair uses; host / port: its address
    UdpPeer(int fd, const std::string& host, int port);
    // sendto() every datagram; a full socket buffer drops the datagram (as a UDP send would
    // under congestion; NACK recovers it).  Returns datagrams sent.
    int send(const std::vector<std::string>& dgrams) const;
    int fd() const { return fd_; }

   private:
    int fd_;
    sockaddr_storage addr_{};
    socklen_t len_ = 0;
};

// packets -> history + SRTP -> socket
int send_rtp_packets(const std::vector<std::string>& raw, SrtpSession& srtp, RtpHistory& hist, const UdpPeer& peer);

}  // namespace net
}  // namespace mx
