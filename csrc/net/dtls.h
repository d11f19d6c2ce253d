// DTLS 1.2 endpoint for DTLS-SRTP (RFC 5764) driven through memory BIOs, so the caller owns
// the UDP socket (one port demultiplexes STUN / DTLS / SRTP, RFC 7983).  A self-signed
// ECDSA P-256 certificate is generated per process; the peer certificate is accepted
// during the handshake and checked afterwards against the SDP a=fingerprint.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

class DtlsEndpoint {
   public:
    explicit DtlsEndpoint(bool server, int mtu = 1200);
    ~DtlsEndpoint();
    DtlsEndpoint(const DtlsEndpoint&) = delete;
    DtlsEndpoint& operator=(const DtlsEndpoint&) = delete;

    // "sha-256 AB:CD:..." of our certificate (for SDP a=fingerprint)
    std::string fingerprint() const;
    // Start the handshake (client sends ClientHello); returns datagrams to send.
    std::vector<std::string> start();
    // Feed one received datagram; returns datagrams to send.
    std::vector<std::string> feed(const std::string& datagram);
    // Retransmission timer; call periodically. Returns datagrams to send.
    std::vector<std::string> tick();
    bool handshake_done() const { return done_; }
    bool failed() const { return failed_; }
    std::string error() const { return err_; }
    // Peer certificate fingerprint, "sha-256 AB:..." (after the handshake).
    std::string peer_fingerprint() const;
    std::string srtp_profile() const;
    // 60 bytes: client key | server key | client salt | server salt
    std::string export_srtp_keys() const;
    // Application data (SCTP for WebRTC data channels, RFC 8261): encrypt one message into
    // DTLS record(s) and return the datagrams to send; empty before the handshake is done.
    std::vector<std::string> write(const std::string& data);
    // Decrypted application-data records received by feed(), in arrival order.
    std::vector<std::string> take_app_data();

   private:
    std::vector<std::string> drain();
    void step();

    void* ctx_ = nullptr;  // SSL_CTX*
    void* ssl_ = nullptr;  // SSL*
    void* rbio_ = nullptr;
    void* wbio_ = nullptr;
    bool server_;
    int mtu_;
    bool done_ = false;
    bool failed_ = false;
    std::string err_;
    std::vector<std::string> app_in_;
};

// Certificate/key shared by all endpoints of the process.
std::string dtls_certificate_fingerprint();

}  // namespace net
}  // namespace mx
