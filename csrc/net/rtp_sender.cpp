#include "rtp_sender.h"

#include <arpa/inet.h>
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

int UdpPeer::send(const std::vector<std::string>& dgrams) const {
    int n = 0;
    for (const std::string& d : dgrams) {
        ssize_t r;
        do {
            r = ::sendto(fd_, d.data(), d.size(), 0, reinterpret_cast<const sockaddr*>(&addr_), len_);
        } while (r < 0 && errno == EINTR);
        if (r >= 0) ++n;
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
