// SRTP / SRTCP with AES_CM_128_HMAC_SHA1_80 (RFC 3711), the profile negotiated by
// DTLS-SRTP with browsers (RFC 5764).  Replaces libsrtp used by GStreamer webrtcbin in
// the reference's selkies pipeline (reference Dockerfile:439-444 installs libsrtp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mx {
namespace net {

class SrtpSession {
   public:
    // master key 16 bytes, master salt 14 bytes
    SrtpSession(const std::string& master_key, const std::string& master_salt);
    ~SrtpSession();
    SrtpSession(const SrtpSession&) = delete;
    SrtpSession& operator=(const SrtpSession&) = delete;

    // Protect one RTP packet (header + payload); returns the SRTP packet.
    std::string protect_rtp(const std::string& rtp);
    // Unprotect; returns empty string on authentication failure / replay.
    std::string unprotect_rtp(const std::string& srtp);
    std::string protect_rtcp(const std::string& rtcp);
    std::string unprotect_rtcp(const std::string& srtcp);

    // Session keys (for tests against RFC 3711 B.3)
    std::string rtp_key() const { return std::string((const char*)k_e_, 16); }
    std::string rtp_salt() const { return std::string((const char*)k_s_, 14); }
    std::string rtp_auth() const { return std::string((const char*)k_a_, 20); }
    std::string rtcp_key() const { return std::string((const char*)c_e_, 16); }

    // Raw AES-CM keystream (RFC 3711 B.2 test vector).
    static std::string aes_cm_keystream(const std::string& key, const std::string& iv16, size_t n);

   private:
    void xor_keystream(const uint8_t* key, const uint8_t* salt, uint32_t ssrc, uint64_t index, uint8_t* data,
                       size_t n) const;
    void hmac80(const uint8_t* key, const uint8_t* data, size_t n, const uint8_t* extra, size_t extra_n,
                uint8_t out[10]) const;

    uint8_t k_e_[16], k_a_[20], k_s_[14];  // SRTP session keys
    uint8_t c_e_[16], c_a_[20], c_s_[14];  // SRTCP session keys
    // sender state
    uint32_t roc_ = 0;
    uint16_t last_seq_ = 0;
    bool have_seq_ = false;
    uint32_t srtcp_index_ = 0;
    // receiver state (single source is enough for our peers)
    uint32_t r_roc_ = 0;
    uint16_t r_seq_ = 0;
    bool r_have_ = false;
    void* cipher_ctx_ = nullptr;  // EVP_CIPHER_CTX*
};

}  // namespace net
}  // namespace mx
