#include "dtls.h"

#include <openssl/bio.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <openssl/srtp.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>

#include <cstdio>
#include <mutex>
#include <stdexcept>

namespace mx {
namespace net {

namespace {

struct Identity {
    EVP_PKEY* key = nullptr;
    X509* cert = nullptr;
};

Identity& identity() {
    static Identity id;
    static std::once_flag once;
    std::call_once(once, [] {
        EVP_PKEY_CTX* pctx = EVP_PKEY_CTX_new_id(EVP_PKEY_EC, nullptr);
        if (!pctx || EVP_PKEY_keygen_init(pctx) <= 0 ||
            EVP_PKEY_CTX_set_ec_paramgen_curve_nid(pctx, NID_X9_62_prime256v1) <= 0 ||
            EVP_PKEY_keygen(pctx, &id.key) <= 0)
            throw std::runtime_error("DTLS: EC key generation failed");
        EVP_PKEY_CTX_free(pctx);
        id.cert = X509_new();
        X509_set_version(id.cert, 2);
        unsigned char serial[8];
        RAND_bytes(serial, sizeof serial);
        ASN1_INTEGER_set(X509_get_serialNumber(id.cert), (long)((serial[0] << 16) | (serial[1] << 8) | serial[2]));
        X509_gmtime_adj(X509_getm_notBefore(id.cert), -86400);
        X509_gmtime_adj(X509_getm_notAfter(id.cert), 30L * 86400);
        X509_set_pubkey(id.cert, id.key);
        X509_NAME* name = X509_get_subject_name(id.cert);
        X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, (const unsigned char*)"mxdesk", -1, -1, 0);
        X509_set_issuer_name(id.cert, name);
        if (!X509_sign(id.cert, id.key, EVP_sha256())) throw std::runtime_error("DTLS: certificate signing failed");
    });
    return id;
}

std::string fp_of(X509* cert) {
    unsigned char md[EVP_MAX_MD_SIZE];
    unsigned int n = 0;
    X509_digest(cert, EVP_sha256(), md, &n);
    std::string s = "sha-256 ";
    char buf[4];
    for (unsigned int i = 0; i < n; ++i) {
        std::snprintf(buf, sizeof buf, i ? ":%02X" : "%02X", md[i]);
        s += buf;
    }
    return s;
}

int accept_any(int, X509_STORE_CTX*) { return 1; }  // verified by fingerprint after the handshake

}  // namespace

std::string dtls_certificate_fingerprint() { return fp_of(identity().cert); }

DtlsEndpoint::DtlsEndpoint(bool server, int mtu) : server_(server), mtu_(mtu) {
    Identity& id = identity();
    SSL_CTX* ctx = SSL_CTX_new(DTLS_method());
    if (!ctx) throw std::runtime_error("DTLS: SSL_CTX_new failed");
    SSL_CTX_set_min_proto_version(ctx, DTLS1_2_VERSION);
    SSL_CTX_use_certificate(ctx, id.cert);
    SSL_CTX_use_PrivateKey(ctx, id.key);
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, accept_any);
    if (SSL_CTX_set_tlsext_use_srtp(ctx, "SRTP_AES128_CM_SHA1_80") != 0)
        throw std::runtime_error("DTLS: use_srtp failed");
    SSL_CTX_set_read_ahead(ctx, 1);
    ctx_ = ctx;
    SSL* ssl = SSL_new(ctx);
    BIO* r = BIO_new(BIO_s_mem());
    BIO* w = BIO_new(BIO_s_mem());
    BIO_set_mem_eof_return(r, -1);
    SSL_set_bio(ssl, r, w);
    SSL_set_options(ssl, SSL_OP_NO_QUERY_MTU);
    DTLS_set_link_mtu(ssl, mtu);
    if (server)
        SSL_set_accept_state(ssl);
    else
        SSL_set_connect_state(ssl);
    ssl_ = ssl;
    rbio_ = r;
    wbio_ = w;
}

DtlsEndpoint::~DtlsEndpoint() {
    if (ssl_) SSL_free((SSL*)ssl_);  // frees the BIOs
    if (ctx_) SSL_CTX_free((SSL_CTX*)ctx_);
}

std::string DtlsEndpoint::fingerprint() const { return dtls_certificate_fingerprint(); }

// Split the memory BIO's byte stream into datagrams at DTLS record boundaries (13-byte
// record header, length in bytes 11..12), packing records up to the MTU.
std::vector<std::string> DtlsEndpoint::drain() {
    std::vector<std::string> out;
    BIO* w = (BIO*)wbio_;
    std::string buf;
    char tmp[4096];
    int n;
    while ((n = BIO_read(w, tmp, sizeof tmp)) > 0) buf.append(tmp, n);
    size_t pos = 0;
    std::string dgram;
    while (pos + 13 <= buf.size()) {
        const size_t len = 13 + (((uint8_t)buf[pos + 11] << 8) | (uint8_t)buf[pos + 12]);
        if (pos + len > buf.size()) break;
        if (!dgram.empty() && dgram.size() + len > (size_t)mtu_) {
            out.push_back(dgram);
            dgram.clear();
        }
        dgram.append(buf, pos, len);
        pos += len;
    }
    if (!dgram.empty()) out.push_back(dgram);
    return out;
}

void DtlsEndpoint::step() {
    SSL* ssl = (SSL*)ssl_;
    if (!done_) {
        const int r = SSL_do_handshake(ssl);
        if (r == 1) {
            done_ = true;
        } else {
            const int e = SSL_get_error(ssl, r);
            if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) {
                failed_ = true;
                char b[256];
                ERR_error_string_n(ERR_get_error(), b, sizeof b);
                err_ = b;
            }
        }
    }
    if (done_) {
        // application data (SCTP packets) that arrived with or after the final flight;
        // SSL_read also processes alerts and renegotiation records
        char tmp[16384];
        int n;
        while ((n = SSL_read(ssl, tmp, sizeof tmp)) > 0) app_in_.emplace_back(tmp, (size_t)n);
    }
}

std::vector<std::string> DtlsEndpoint::start() {
    step();
    return drain();
}

std::vector<std::string> DtlsEndpoint::feed(const std::string& d) {
    BIO_write((BIO*)rbio_, d.data(), (int)d.size());
    step();
    return drain();
}

std::vector<std::string> DtlsEndpoint::tick() {
    if (!done_ && DTLSv1_handle_timeout((SSL*)ssl_) > 0) return drain();
    return {};
}

std::vector<std::string> DtlsEndpoint::write(const std::string& data) {
    if (!done_ || failed_ || data.empty()) return {};
    if (SSL_write((SSL*)ssl_, data.data(), (int)data.size()) <= 0) return {};
    return drain();
}

std::vector<std::string> DtlsEndpoint::take_app_data() {
    std::vector<std::string> v;
    v.swap(app_in_);
    return v;
}

std::string DtlsEndpoint::peer_fingerprint() const {
    X509* c = SSL_get1_peer_certificate((SSL*)ssl_);
    if (!c) return {};
    std::string s = fp_of(c);
    X509_free(c);
    return s;
}

std::string DtlsEndpoint::srtp_profile() const {
    SRTP_PROTECTION_PROFILE* p = SSL_get_selected_srtp_profile((SSL*)ssl_);
    return p ? std::string(p->name) : std::string();
}

std::string DtlsEndpoint::export_srtp_keys() const {
    if (!done_) throw std::logic_error("DTLS handshake not complete");
    unsigned char km[60];
    static const char label[] = "EXTRACTOR-dtls_srtp";
    if (SSL_export_keying_material((SSL*)ssl_, km, sizeof km, label, sizeof(label) - 1, nullptr, 0, 0) != 1)
        throw std::runtime_error("DTLS: keying material export failed");
    return std::string((const char*)km, sizeof km);
}

}  // namespace net
}  // namespace mx
