#include "srtp.h"

#include <openssl/evp.h>
#include <openssl/hmac.h>

#include <cstring>
#include <stdexcept>

namespace mx {
namespace net {

namespace {

void aes_ecb_blocks(EVP_CIPHER_CTX* ctx, const uint8_t* key, const uint8_t* in, uint8_t* out, size_t nblocks) {
    int len = 0;
    if (EVP_EncryptInit_ex(ctx, EVP_aes_128_ecb(), nullptr, key, nullptr) != 1)
        throw std::runtime_error("AES init failed");
    EVP_CIPHER_CTX_set_padding(ctx, 0);
    if (EVP_EncryptUpdate(ctx, out, &len, in, (int)(16 * nblocks)) != 1) throw std::runtime_error("AES failed");
}

// AES-CM keystream of n bytes for a 128-bit initial counter block (low 16 bits count).
void keystream(EVP_CIPHER_CTX* ctx, const uint8_t* key, const uint8_t iv[16], uint8_t* out, size_t n) {
    if (n == 0) return;
    const size_t nb = (n + 15) / 16;
    std::vector<uint8_t> ctr(nb * 16), ks(nb * 16);
    for (size_t b = 0; b < nb; ++b) {
        std::memcpy(&ctr[b * 16], iv, 16);
        // add b to the 128-bit big-endian counter (only low bytes change in practice)
        uint32_t carry = (uint32_t)b;
        for (int i = 15; i >= 0 && carry; --i) {
            const uint32_t v = ctr[b * 16 + i] + (carry & 0xff);
            ctr[b * 16 + i] = (uint8_t)v;
            carry = (carry >> 8) + (v >> 8);
        }
    }
    aes_ecb_blocks(ctx, key, ctr.data(), ks.data(), nb);
    std::memcpy(out, ks.data(), n);
}

// RFC 3711 4.3.1 key derivation (key_derivation_rate = 0).
void derive(EVP_CIPHER_CTX* ctx, const uint8_t* mkey, const uint8_t* msalt, uint8_t label, uint8_t* out, size_t n) {
    uint8_t iv[16] = {0};
    std::memcpy(iv, msalt, 14);
    iv[7] ^= label;  // key_id = label || 48-bit zero index, aligned to the low end of the 112-bit salt
    keystream(ctx, mkey, iv, out, n);
}

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

size_t rtp_header_len(const std::string& p) {
    if (p.size() < 12) throw std::invalid_argument("short RTP packet");
    const uint8_t* b = (const uint8_t*)p.data();
    size_t len = 12 + 4 * (b[0] & 0x0f);
    if (b[0] & 0x10) {  // header extension
        if (p.size() < len + 4) throw std::invalid_argument("bad RTP extension");
        len += 4 + 4 * be16(b + len + 2);
    }
    if (len > p.size()) throw std::invalid_argument("bad RTP header");
    return len;
}

}  // namespace

SrtpSession::SrtpSession(const std::string& master_key, const std::string& master_salt) {
    if (master_key.size() != 16 || master_salt.size() != 14)
        throw std::invalid_argument("SRTP needs a 16-byte master key and 14-byte master salt");
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    cipher_ctx_ = ctx;
    const uint8_t* mk = (const uint8_t*)master_key.data();
    const uint8_t* ms = (const uint8_t*)master_salt.data();
    derive(ctx, mk, ms, 0, k_e_, 16);
    derive(ctx, mk, ms, 1, k_a_, 20);
    derive(ctx, mk, ms, 2, k_s_, 14);
    derive(ctx, mk, ms, 3, c_e_, 16);
    derive(ctx, mk, ms, 4, c_a_, 20);
    derive(ctx, mk, ms, 5, c_s_, 14);
}

SrtpSession::~SrtpSession() { EVP_CIPHER_CTX_free((EVP_CIPHER_CTX*)cipher_ctx_); }

std::string SrtpSession::aes_cm_keystream(const std::string& key, const std::string& iv16, size_t n) {
    if (key.size() != 16 || iv16.size() != 16) throw std::invalid_argument("key/iv must be 16 bytes");
    EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
    std::string out(n, '\0');
    keystream(ctx, (const uint8_t*)key.data(), (const uint8_t*)iv16.data(), (uint8_t*)&out[0], n);
    EVP_CIPHER_CTX_free(ctx);
    return out;
}

void SrtpSession::xor_keystream(const uint8_t* key, const uint8_t* salt, uint32_t ssrc, uint64_t index,
                                uint8_t* data, size_t n) const {
    if (n == 0) return;
    // IV = (salt * 2^16) XOR (SSRC * 2^64) XOR (index * 2^16)
    uint8_t iv[16] = {0};
    std::memcpy(iv, salt, 14);
    iv[4] ^= (uint8_t)(ssrc >> 24);
    iv[5] ^= (uint8_t)(ssrc >> 16);
    iv[6] ^= (uint8_t)(ssrc >> 8);
    iv[7] ^= (uint8_t)ssrc;
    for (int i = 0; i < 6; ++i) iv[8 + i] ^= (uint8_t)(index >> (40 - 8 * i));
    std::vector<uint8_t> ks(n);
    keystream((EVP_CIPHER_CTX*)cipher_ctx_, key, iv, ks.data(), n);
    for (size_t i = 0; i < n; ++i) data[i] ^= ks[i];
}

void SrtpSession::hmac80(const uint8_t* key, const uint8_t* data, size_t n, const uint8_t* extra, size_t extra_n,
                         uint8_t out[10]) const {
    uint8_t md[EVP_MAX_MD_SIZE];
    unsigned int mdlen = 0;
    HMAC_CTX* h = HMAC_CTX_new();
    HMAC_Init_ex(h, key, 20, EVP_sha1(), nullptr);
    HMAC_Update(h, data, n);
    if (extra_n) HMAC_Update(h, extra, extra_n);
    HMAC_Final(h, md, &mdlen);
    HMAC_CTX_free(h);
    std::memcpy(out, md, 10);
}

std::string SrtpSession::protect_rtp(const std::string& rtp) {
    const size_t hl = rtp_header_len(rtp);
    std::string out = rtp;
    uint8_t* b = (uint8_t*)&out[0];
    const uint16_t seq = be16(b + 2);
    const uint32_t ssrc = be32(b + 8);
    // Sender-side index: advance ROC on forward wrap; a retransmission of a packet sent
    // before the last wrap keeps its original (previous) ROC.
    uint32_t v = roc_;
    if (!have_seq_) {
        last_seq_ = seq;
        have_seq_ = true;
    } else {
        const int16_t d = (int16_t)(uint16_t)(seq - last_seq_);
        if (d > 0) {
            if (seq < last_seq_) v = ++roc_;
            last_seq_ = seq;
        } else if (d < 0 && seq > last_seq_) {
            v = roc_ - 1;
        }
    }
    const uint64_t index = ((uint64_t)v << 16) | seq;
    xor_keystream(k_e_, k_s_, ssrc, index, b + hl, out.size() - hl);
    const uint8_t roc_be[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    uint8_t tag[10];
    hmac80(k_a_, (const uint8_t*)out.data(), out.size(), roc_be, 4, tag);
    out.append((const char*)tag, 10);
    return out;
}

std::string SrtpSession::unprotect_rtp(const std::string& srtp) {
    if (srtp.size() < 12 + 10) return {};
    std::string pkt = srtp.substr(0, srtp.size() - 10);
    const size_t hl = rtp_header_len(pkt);
    uint8_t* b = (uint8_t*)&pkt[0];
    const uint16_t seq = be16(b + 2);
    const uint32_t ssrc = be32(b + 8);
    // RFC 3711 Appendix A index estimation
    uint32_t v = r_roc_;
    if (r_have_) {
        if (r_seq_ < 0x8000) {
            if ((int)seq - (int)r_seq_ > 0x8000) v = r_roc_ - 1;
        } else if ((int)r_seq_ - 0x8000 > (int)seq) {
            v = r_roc_ + 1;
        }
    }
    const uint8_t roc_be[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    uint8_t tag[10];
    hmac80(k_a_, (const uint8_t*)pkt.data(), pkt.size(), roc_be, 4, tag);
    if (std::memcmp(tag, srtp.data() + srtp.size() - 10, 10) != 0) return {};
    const uint64_t index = ((uint64_t)v << 16) | seq;
    xor_keystream(k_e_, k_s_, ssrc, index, b + hl, pkt.size() - hl);
    if (!r_have_ || v > r_roc_ || (v == r_roc_ && seq > r_seq_)) {
        r_roc_ = v;
        r_seq_ = seq;
    }
    r_have_ = true;
    return pkt;
}

std::string SrtpSession::protect_rtcp(const std::string& rtcp) {
    if (rtcp.size() < 8) throw std::invalid_argument("short RTCP packet");
    std::string out = rtcp;
    uint8_t* b = (uint8_t*)&out[0];
    const uint32_t ssrc = be32(b + 4);
    const uint32_t idx = (srtcp_index_++) & 0x7fffffff;
    xor_keystream(c_e_, c_s_, ssrc, idx, b + 8, out.size() - 8);
    const uint32_t e_idx = 0x80000000u | idx;
    const char eb[4] = {(char)(e_idx >> 24), (char)(e_idx >> 16), (char)(e_idx >> 8), (char)e_idx};
    out.append(eb, 4);
    uint8_t tag[10];
    hmac80(c_a_, (const uint8_t*)out.data(), out.size(), nullptr, 0, tag);
    out.append((const char*)tag, 10);
    return out;
}

std::string SrtpSession::unprotect_rtcp(const std::string& srtcp) {
    if (srtcp.size() < 8 + 4 + 10) return {};
    const size_t n = srtcp.size() - 10;
    uint8_t tag[10];
    hmac80(c_a_, (const uint8_t*)srtcp.data(), n, nullptr, 0, tag);
    if (std::memcmp(tag, srtcp.data() + n, 10) != 0) return {};
    std::string pkt = srtcp.substr(0, n - 4);
    const uint32_t e_idx = be32((const uint8_t*)srtcp.data() + n - 4);
    if (e_idx & 0x80000000u) {
        uint8_t* b = (uint8_t*)&pkt[0];
        xor_keystream(c_e_, c_s_, be32(b + 4), e_idx & 0x7fffffff, b + 8, pkt.size() - 8);
    }
    return pkt;
}

}  // namespace net
}  // namespace mx
