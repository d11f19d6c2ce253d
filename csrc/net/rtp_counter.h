// Native receive side of the density harness's "lite" WebRTC viewer (tools/bench_density.py
// --client native): after the Python viewer finished ICE and the DTLS-SRTP
// handshake, the UDP socket is handed to this loop, which drains it with recvmmsg() in batches and
// counts access units from the plaintext RTP headers (SRTP encrypts only the payload): a frame is
// the packets of one RTP timestamp, complete when the marker packet arrives with every sequence
// number in between.  The last RTCP packets (the sender reports that map RTP time to wall time)
// are kept raw for the caller to decrypt.  Runs with the GIL released; no per-packet Python work,
// so the viewers no longer compete with the serve processes for the host CPUs.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

struct RtpFrameCount {
    std::vector<uint32_t> rtp_ts;       // RTP timestamp of every complete frame
    std::vector<int64_t> arrival_us;    // CLOCK_MONOTONIC microseconds when it completed
    std::vector<double> arrival_wall;   // CLOCK_REALTIME seconds (time.time()) when it completed
    std::vector<std::string> rtcp;      // the last kRtcpKeep RTCP datagrams, raw (SRTCP)
    uint64_t packets = 0;               // RTP video packets
    uint64_t lost = 0;                  // sequence numbers skipped
    uint64_t datagrams = 0;
    bool timed_out = false;
};

// State of the frame being received (the Python loop's, when it hands over mid-frame).
struct RtpLiteState {
    int64_t ts = -1;    // RTP timestamp of the frame in progress (-1: none)
    int32_t next = -1;  // next expected sequence number (-1: none yet)
    bool ok = true;     // every packet of the frame in progress arrived in order
};

// Receive on `fd` (a connected, non-blocking UDP socket) until `n_frames` complete frames or
// `timeout_s` seconds.  Audio (payload type 0) and DTLS / STUN datagrams are skipped.
RtpFrameCount count_rtp_frames(int fd, int n_frames, double timeout_s, RtpLiteState state = {});

}  // namespace net
}  // namespace mx
