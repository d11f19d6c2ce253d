#include "rtp_sender.h"

#include <arpa/inet.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace mx {
namespace net {

UdpPeer::UdpPeer(int fd, const std::string& host, int port) : fd_(fd) {
    std::memset(&addr_, 0, sizeof addr_);
    sockaddr_in* a4 = reinterpret_cast<sockaddr_in*>(&addr_);
    sockaddr_in6* a6 = reinterpret_cast<sockaddr_in6*>(&addr_);
    if (inet_pton(AF_INET, host.c_str(), &a4->sin_addr) == 1) {
        a4->sin_family = AF_INET;
        a4->sin_port = htons((uint16_t)port);
        len_ = sizeof(sockaddr_in);
    } else if (inet_pton(AF_INET6, host.c_str(), &a6->sin6_addr) == 1) {
        a6->sin6_family = AF_INET6;
        a6->sin6_port = htons((uint16_t)port);
        len_ = sizeof(sockaddr_in6);
    } else {
        throw std::invalid_argument("UdpPeer: not a numeric address: " + host);
    }
}

// One sendmmsg per up to kBatch datagrams (an access unit's packets in one or two system calls
// instead of one sendto each: the per-packet syscall was a visible share of a serve process's CPU
// at density).  A datagram the socket refuses (e.g. EAGAIN on a full non-blocking buffer) is
// dropped and the rest still go out, as with one sendto per packet; the return value counts the
// datagrams sent.
int UdpPeer::send(const std::vector<std::string>& dgrams) const {
    constexpr size_t kBatch = 64;
    mmsghdr msgs[kBatch];
    iovec iov[kBatch];
    int n = 0;
    size_t i = 0;
    while (i < dgrams.size()) {
        const size_t m = std::min(kBatch, dgrams.size() - i);
        for (size_t k = 0; k < m; ++k) {
            const std::string& d = dgrams[i + k];
            iov[k].iov_base = const_cast<char*>(d.data());
            iov[k].iov_len = d.size();
            std::memset(&msgs[k], 0, sizeof msgs[k]);
            msgs[k].msg_hdr.msg_name = const_cast<sockaddr_storage*>(&addr_);
            msgs[k].msg_hdr.msg_namelen = len_;
            msgs[k].msg_hdr.msg_iov = &iov[k];
            msgs[k].msg_hdr.msg_iovlen = 1;
        }
        const int r = ::sendmmsg(fd_, msgs, (unsigned)m, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            ++i;  // the first datagram of the batch was refused: drop it, send the rest
            continue;
        }
        n += r;
        i += r > 0 ? (size_t)r : 1;  // r < m: the next call reports (and drops) the datagram that stopped it
    }
    return n;
}

int send_rtp_packets(const std::vector<std::string>& raw, SrtpSession& srtp, RtpHistory& hist, const UdpPeer& peer) {
    std::vector<std::string> out;
    out.reserve(raw.size());
    for (const std::string& p : raw) {
        if (p.size() < 12) continue;
        const uint16_t seq = (uint16_t)(((uint8_t)p[2] << 8) | (uint8_t)p[3]);
        hist.put(seq, p);
        out.push_back(srtp.protect_rtp(p));
    }
    return peer.send(out);
}

}  // namespace net
}  // namespace mx
