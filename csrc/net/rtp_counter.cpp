// recvmmsg() receive loop of the native density viewer (rtp_counter.h).
#include "rtp_counter.h"

#include <poll.h>
#include <sys/socket.h>
#include <time.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

namespace mx {
namespace net {

namespace {
constexpr int kBatch = 64;         // datagrams per recvmmsg()
constexpr size_t kDgram = 2048;    // largest datagram kept (RTP packets are <= ~1200 bytes)
constexpr size_t kRtcpKeep = 8;

int64_t mono_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (int64_t)t.tv_sec * 1000000 + t.tv_nsec / 1000;
}
double wall_s() {
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    return (double)t.tv_sec + t.tv_nsec * 1e-9;
}
}  // namespace

RtpFrameCount count_rtp_frames(int fd, int n_frames, double timeout_s, RtpLiteState st) {
    RtpFrameCount out;
    std::vector<uint8_t> buf((size_t)kBatch * kDgram);
    mmsghdr msgs[kBatch];
    iovec iov[kBatch];
    const int64_t deadline = mono_us() + (int64_t)(timeout_s * 1e6);
    while ((int)out.rtp_ts.size() < n_frames) {
        const int64_t now = mono_us();
        if (now >= deadline) {
            out.timed_out = true;
            break;
        }
        pollfd pfd{fd, POLLIN, 0};
        const int wait_ms = (int)std::min<int64_t>(50, (deadline - now) / 1000 + 1);
        const int pr = poll(&pfd, 1, wait_ms);
        if (pr < 0 && errno != EINTR) break;
        if (pr <= 0) continue;
        for (int i = 0; i < kBatch; ++i) {
            iov[i].iov_base = buf.data() + (size_t)i * kDgram;
            iov[i].iov_len = kDgram;
            std::memset(&msgs[i], 0, sizeof msgs[i]);
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
        }
        const int n = recvmmsg(fd, msgs, kBatch, MSG_DONTWAIT, nullptr);
        if (n <= 0) continue;
        const int64_t t_us = mono_us();  // one arrival stamp per batch
        const double t_wall = wall_s();
        for (int i = 0; i < n; ++i) {
            const uint8_t* d = buf.data() + (size_t)i * kDgram;
            const size_t len = msgs[i].msg_len;
            ++out.datagrams;
            if (len < 12 || d[0] < 128 || d[0] > 191) continue;  // not RTP / RTCP (STUN, DTLS)
            if (d[1] >= 192 && d[1] <= 223) {                    // RTCP
                if (out.rtcp.size() == kRtcpKeep) out.rtcp.erase(out.rtcp.begin());
                out.rtcp.emplace_back(reinterpret_cast<const char*>(d), len);
                continue;
            }
            if ((d[1] & 0x7f) == 0) continue;  // PCMU audio
            const int seq = (d[2] << 8) | d[3];
            const int64_t ts = ((int64_t)d[4] << 24) | (d[5] << 16) | (d[6] << 8) | d[7];
            ++out.packets;
            if (ts != st.ts) {  // a new frame begins
                st.ts = ts;
                st.ok = st.next < 0 || seq == st.next;
            } else if (seq != st.next) {
                st.ok = false;
            }
            if (st.next >= 0 && seq != st.next) {
                const int gap = (seq - st.next) & 0xffff;
                if (gap < 0x8000) out.lost += (uint64_t)gap;
            }
            st.next = (seq + 1) & 0xffff;
            if (d[1] & 0x80) {  // marker: the frame's last packet
                if (st.ok && (int)out.rtp_ts.size() < n_frames) {
                    out.rtp_ts.push_back((uint32_t)ts);
                    out.arrival_us.push_back(t_us);
                    out.arrival_wall.push_back(t_wall);
                }
                st.ts = -1;
            }
        }
    }
    return out;
}

}  // namespace net
}  // namespace mx
