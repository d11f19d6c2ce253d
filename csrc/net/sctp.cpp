#include "sctp.h"

#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace mx {
namespace net {

namespace {

enum : uint8_t {
    C_DATA = 0, C_INIT = 1, C_INIT_ACK = 2, C_SACK = 3, C_HEARTBEAT = 4, C_HEARTBEAT_ACK = 5, C_ABORT = 6,
    C_SHUTDOWN = 7, C_SHUTDOWN_ACK = 8, C_ERROR = 9, C_COOKIE_ECHO = 10, C_COOKIE_ACK = 11,
    C_SHUTDOWN_COMPLETE = 14, C_RECONFIG = 130, C_FORWARD_TSN = 192,
};
enum : uint16_t {
    P_STATE_COOKIE = 7, P_OUT_RESET = 13, P_IN_RESET = 14, P_RECONFIG_RESP = 16, P_SUPPORTED_EXT = 0x8008,
    P_FORWARD_TSN_SUPPORTED = 0xC000,
};
constexpr uint8_t F_E = 1, F_B = 2, F_U = 4;
constexpr uint32_t kMtu = SctpAssociation::kMaxPacket;
constexpr uint32_t kRtoMin = 200, kRtoMax = 10000, kRtoInit = 1000;
constexpr int kMaxAssocRetrans = 10, kMaxInitRetrans = 8;
constexpr int64_t kCookieLifeMs = 60000;
constexpr size_t kCookieBody = 4 * 5 + 1 + 8;  // tags, TSNs, rwnd, ext, timestamp
constexpr size_t kCookieLen = kCookieBody + 32;  // + HMAC-SHA256

inline bool lt(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
inline bool le(uint32_t a, uint32_t b) { return (int32_t)(a - b) <= 0; }
inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }
inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3];
}
inline void put8(std::string& s, uint8_t v) { s.push_back((char)v); }
inline void put16(std::string& s, uint16_t v) {
    s.push_back((char)(v >> 8));
    s.push_back((char)v);
}
inline void put32(std::string& s, uint32_t v) {
    put16(s, (uint16_t)(v >> 16));
    put16(s, (uint16_t)v);
}
inline void put64(std::string& s, uint64_t v) {
    put32(s, (uint32_t)(v >> 32));
    put32(s, (uint32_t)v);
}
inline size_t pad4(size_t n) { return (n + 3) & ~(size_t)3; }

std::string chunk(uint8_t type, uint8_t flags, const std::string& value) {
    std::string c;
    c.reserve(4 + value.size() + 3);
    put8(c, type);
    put8(c, flags);
    put16(c, (uint16_t)(4 + value.size()));
    c += value;
    return c;
}

std::string param(uint16_t type, const std::string& value) {
    std::string p;
    put16(p, type);
    put16(p, (uint16_t)(4 + value.size()));
    p += value;
    p.resize(pad4(p.size()), '\0');
    return p;
}

uint32_t rand_nonzero() {
    uint32_t v = 0;
    while (v == 0)
        if (RAND_bytes((unsigned char*)&v, sizeof v) != 1) throw std::runtime_error("SCTP: RAND_bytes failed");
    return v;
}

struct Crc32cTable {
    uint32_t t[8][256];
    Crc32cTable() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1)));
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 255];
    }
};
const Crc32cTable& crc_table() {
    static const Crc32cTable tab;
    return tab;
}

}  // namespace

uint32_t crc32c(const void* data, size_t n) {
    const Crc32cTable& T = crc_table();
    const uint8_t* p = (const uint8_t*)data;
    uint32_t c = 0xFFFFFFFFu;
    while (n >= 8) {  // slicing-by-8
        const uint32_t lo = c ^ ((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
        const uint32_t hi = (uint32_t)p[4] | (uint32_t)p[5] << 8 | (uint32_t)p[6] << 16 | (uint32_t)p[7] << 24;
        c = T.t[7][lo & 255] ^ T.t[6][(lo >> 8) & 255] ^ T.t[5][(lo >> 16) & 255] ^ T.t[4][lo >> 24] ^
            T.t[3][hi & 255] ^ T.t[2][(hi >> 8) & 255] ^ T.t[1][(hi >> 16) & 255] ^ T.t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 255];
    return ~c;
}

// ====================================================================== association
SctpAssociation::SctpAssociation(uint16_t local_port, uint16_t remote_port, size_t max_message)
    : lport_(local_port), rport_(remote_port), max_message_(max_message) {
    if (RAND_bytes(secret_, sizeof secret_) != 1) throw std::runtime_error("SCTP: RAND_bytes failed");
    rto_ = kRtoInit;
}

int64_t SctpAssociation::now() const {
    if (clock_ >= 0) return clock_;
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Common header + chunks (each padded to 4 bytes); CRC-32C over the packet with a zero
// checksum field, stored least-significant byte first as the RFC 4960 App. B reference
// code (and every deployed stack) does.
std::string SctpAssociation::build(const std::vector<std::string>& chunks, uint32_t vtag) const {
    std::string p;
    size_t n = 12;
    for (const auto& c : chunks) n += pad4(c.size());
    p.reserve(n);
    put16(p, lport_);
    put16(p, rport_);
    put32(p, vtag);
    put32(p, 0);
    for (const auto& c : chunks) {
        p += c;
        p.resize(pad4(p.size()), '\0');
    }
    const uint32_t crc = crc32c(p.data(), p.size());
    p[8] = (char)(crc & 255);
    p[9] = (char)((crc >> 8) & 255);
    p[10] = (char)((crc >> 16) & 255);
    p[11] = (char)(crc >> 24);
    return p;
}

std::string SctpAssociation::make_init_chunk(uint8_t type, uint32_t tag, uint32_t itsn,
                                             const std::string& cookie) const {
    std::string v;
    put32(v, tag);
    put32(v, kRwnd);
    put16(v, 65535);  // outbound streams
    put16(v, 65535);  // max inbound streams
    put32(v, itsn);
    v += param(P_SUPPORTED_EXT, std::string{(char)C_FORWARD_TSN, (char)C_RECONFIG});
    v += param(P_FORWARD_TSN_SUPPORTED, "");
    if (!cookie.empty()) v += param(P_STATE_COOKIE, cookie);
    return chunk(type, 0, v);
}

std::string SctpAssociation::make_cookie(uint32_t peer_tag, uint32_t peer_itsn, uint32_t peer_rwnd, uint32_t my_tag,
                                         uint32_t my_itsn, uint8_t ext) const {
    std::string c;
    put32(c, peer_tag);
    put32(c, peer_itsn);
    put32(c, peer_rwnd);
    put32(c, my_tag);
    put32(c, my_itsn);
    put8(c, ext);
    put64(c, (uint64_t)now());
    unsigned char mac[32];
    unsigned int ml = 0;
    HMAC(EVP_sha256(), secret_, sizeof secret_, (const unsigned char*)c.data(), c.size(), mac, &ml);
    c.append((const char*)mac, 32);
    return c;
}

void SctpAssociation::fail(const std::string& why) {
    err_ = why;
    state_ = State::Aborted;
    t1_deadline_ = t3_deadline_ = t2_deadline_ = reconf_deadline_ = -1;
}

void SctpAssociation::enter_established() {
    state_ = State::Established;
    t1_deadline_ = -1;
    errors_ = 0;
    rto_ = have_rtt_ ? rto_ : kRtoInit;
    cwnd_ = std::min(4 * kMtu, std::max(2 * kMtu, 4380u));
    ssthresh_ = peer_rwnd_;
}

std::vector<std::string> SctpAssociation::connect() {
    if (state_ != State::Closed) throw std::logic_error("SCTP: connect() on an open association");
    my_tag_ = rand_nonzero();
    my_itsn_ = rand_nonzero();
    next_tsn_ = my_itsn_;
    cum_acked_ = ack_point_ = my_itsn_ - 1;
    my_reconf_seq_ = my_itsn_;
    state_ = State::CookieWait;
    t1_tries_ = 0;
    t1_deadline_ = now() + rto_;
    return {build({make_init_chunk(C_INIT, my_tag_, my_itsn_, "")}, 0)};
}

std::vector<std::string> SctpAssociation::feed(const std::string& packet) {
    std::vector<std::string> out;
    if (packet.size() < 16 || (packet.size() & 3)) return out;
    stats_.packets_in++;
    const uint8_t* p = (const uint8_t*)packet.data();
    {
        std::string z = packet;
        z[8] = z[9] = z[10] = z[11] = 0;
        const uint32_t crc = crc32c(z.data(), z.size());
        const uint32_t got = (uint32_t)p[8] | (uint32_t)p[9] << 8 | (uint32_t)p[10] << 16 | (uint32_t)p[11] << 24;
        if (crc != got) {
            stats_.bad_checksum++;
            return out;
        }
    }
    if (rd16(p) != rport_ || rd16(p + 2) != lport_) return out;
    const uint32_t vtag = rd32(p + 4);
    const uint8_t first = p[12];
    // verification tag rules (RFC 4960 8.5 / 8.5.1)
    bool ok;
    if (first == C_INIT)
        ok = vtag == 0;
    else if (first == C_COOKIE_ECHO)
        ok = true;  // checked against the tag inside the cookie
    else if ((first == C_ABORT || first == C_SHUTDOWN_COMPLETE) && (p[13] & 1))
        ok = vtag == peer_tag_ && peer_tag_ != 0;
    else
        ok = vtag == my_tag_ && my_tag_ != 0;
    if (!ok) {
        stats_.bad_tag++;
        return out;
    }
    cur_vtag_ = vtag;
    bool sack_needed = false, stop = false;
    size_t off = 12;
    while (!stop && off + 4 <= packet.size()) {
        const uint8_t type = p[off], flags = p[off + 1];
        const size_t len = rd16(p + off + 2);
        if (len < 4 || off + len > packet.size()) break;
        if (type == C_INIT && off != 12) break;  // INIT must be alone
        on_chunk(type, flags, p + off + 4, len - 4, out, sack_needed, stop);
        off += pad4(len);
    }
    if (sack_needed) sack_pending_ = true;
    if (state_ == State::Aborted) return out;
    for (auto& s : flush()) out.push_back(std::move(s));
    return out;
}

void SctpAssociation::on_chunk(uint8_t type, uint8_t flags, const uint8_t* v, size_t n,
                               std::vector<std::string>& out, bool& sack_needed, bool& stop) {
    const bool data_ok = state_ == State::Established || state_ == State::ShutdownPending ||
                         state_ == State::ShutdownSent;
    switch (type) {
        case C_DATA:
            if (data_ok) {
                on_data(flags, v, n);
                sack_needed = true;
            }
            break;
        case C_INIT:
            on_init(v, n, false, out);
            stop = true;
            break;
        case C_INIT_ACK:
            if (state_ == State::CookieWait) on_init(v, n, true, out);
            break;
        case C_SACK:
            if (state_ != State::Closed && state_ != State::CookieWait && state_ != State::CookieEchoed) on_sack(v, n);
            break;
        case C_HEARTBEAT:
            ctrl_.push_back(chunk(C_HEARTBEAT_ACK, 0, std::string((const char*)v, n)));
            break;
        case C_ABORT:
            fail("peer aborted the association");
            stop = true;
            break;
        case C_SHUTDOWN:
            if (n >= 4 && (state_ == State::Established || state_ == State::ShutdownPending ||
                           state_ == State::ShutdownSent)) {
                std::string s;
                put32(s, rd32(v));
                put32(s, peer_rwnd_);
                put32(s, 0);
                on_sack((const uint8_t*)s.data(), s.size());
                if (state_ != State::ShutdownSent) state_ = State::ShutdownReceived;
            }
            break;
        case C_SHUTDOWN_ACK:
            if (state_ == State::ShutdownSent) {
                out.push_back(build({chunk(C_SHUTDOWN_COMPLETE, 0, "")}, peer_tag_));
                state_ = State::Closed;
                t2_deadline_ = t3_deadline_ = -1;
            }
            break;
        case C_SHUTDOWN_COMPLETE:
            if (state_ == State::ShutdownAckSent) {
                state_ = State::Closed;
                t2_deadline_ = t3_deadline_ = -1;
            }
            break;
        case C_COOKIE_ECHO:
            on_cookie_echo(v, n, out);
            break;
        case C_COOKIE_ACK:
            if (state_ == State::CookieEchoed) enter_established();
            break;
        case C_ERROR:
            break;
        case C_FORWARD_TSN:
            if (data_ok) {
                on_forward_tsn(v, n);
                sack_needed = true;
            }
            break;
        case C_RECONFIG:
            if (data_ok) on_reconfig(v, n, out);
            break;
        default:
            // unrecognised: the two high bits say whether to skip it or stop (RFC 4960 3.2)
            if ((type >> 6) < 2) stop = true;
            break;
    }
}

void SctpAssociation::on_init(const uint8_t* v, size_t n, bool ack, std::vector<std::string>& out) {
    if (n < 16) return;
    const uint32_t tag = rd32(v), rwnd = rd32(v + 4), itsn = rd32(v + 12);
    if (tag == 0) return;
    uint8_t ext = 0;
    std::string cookie;
    for (size_t o = 16; o + 4 <= n;) {
        const uint16_t pt = rd16(v + o), pl = rd16(v + o + 2);
        if (pl < 4 || o + pl > n) break;
        const uint8_t* pv = v + o + 4;
        if (pt == P_SUPPORTED_EXT) {
            for (size_t k = 0; k < (size_t)pl - 4; ++k) {
                if (pv[k] == C_FORWARD_TSN) ext |= 1;
                if (pv[k] == C_RECONFIG) ext |= 2;
            }
        } else if (pt == P_FORWARD_TSN_SUPPORTED) {
            ext |= 1;
        } else if (pt == P_STATE_COOKIE) {
            cookie.assign((const char*)pv, pl - 4);
        }
        o += pad4(pl);
    }
    if (!ack) {
        // Passive open stays stateless: everything needed later travels in the signed cookie.
        // An INIT crossing our own (collision, RFC 4960 5.2.1) is answered with our tags.
        uint32_t mt, mi;
        if (state_ == State::CookieWait || state_ == State::CookieEchoed) {
            mt = my_tag_;
            mi = my_itsn_;
        } else {
            mt = rand_nonzero();
            mi = rand_nonzero();
        }
        const std::string ck = make_cookie(tag, itsn, rwnd, mt, mi, ext);
        out.push_back(build({make_init_chunk(C_INIT_ACK, mt, mi, ck)}, tag));
        stats_.packets_out++;
        return;
    }
    if (cookie.empty()) {
        fail("INIT ACK without a state cookie");
        return;
    }
    peer_tag_ = tag;
    peer_itsn_ = itsn;
    peer_rwnd_ = rwnd;
    peer_prsctp_ = ext & 1;
    peer_reconfig_ = ext & 2;
    peer_cum_ = itsn - 1;
    peer_reconf_seq_ = itsn;
    cookie_ = cookie;
    state_ = State::CookieEchoed;
    t1_tries_ = 0;
    t1_deadline_ = now() + rto_;
    out.push_back(build({chunk(C_COOKIE_ECHO, 0, cookie_)}, peer_tag_));
    stats_.packets_out++;
}

void SctpAssociation::on_cookie_echo(const uint8_t* v, size_t n, std::vector<std::string>& out) {
    if (n != kCookieLen) return;
    unsigned char mac[32];
    unsigned int ml = 0;
    HMAC(EVP_sha256(), secret_, sizeof secret_, v, kCookieBody, mac, &ml);
    if (CRYPTO_memcmp(mac, v + kCookieBody, 32) != 0) return;
    const uint32_t ptag = rd32(v), pitsn = rd32(v + 4), prwnd = rd32(v + 8), mtag = rd32(v + 12), mitsn = rd32(v + 16);
    const uint8_t ext = v[20];
    const int64_t ts = (int64_t)((uint64_t)rd32(v + 21) << 32 | rd32(v + 25));
    if (cur_vtag_ != mtag) return;
    if (now() - ts > kCookieLifeMs) return;  // stale cookie
    const bool same = ptag == peer_tag_ && mtag == my_tag_;
    if (state_ == State::Established && same) {  // our COOKIE ACK was lost
        ctrl_.push_back(chunk(C_COOKIE_ACK, 0, ""));
        return;
    }
    if ((state_ == State::CookieWait || state_ == State::CookieEchoed) && mtag == my_tag_) {
        // collision: both sides' handshakes resolve to the same pair of tags
    } else if (state_ != State::Closed) {
        return;  // restarts are not supported; keep the current association
    } else {
        my_tag_ = mtag;
        my_itsn_ = mitsn;
        next_tsn_ = mitsn;
        cum_acked_ = ack_point_ = mitsn - 1;
        my_reconf_seq_ = mitsn;
    }
    peer_tag_ = ptag;
    peer_itsn_ = pitsn;
    peer_rwnd_ = prwnd;
    peer_prsctp_ = ext & 1;
    peer_reconfig_ = ext & 2;
    peer_cum_ = pitsn - 1;
    peer_reconf_seq_ = pitsn;
    enter_established();
    ctrl_.push_back(chunk(C_COOKIE_ACK, 0, ""));
    (void)out;
}

// ---------------------------------------------------------------------- receive side
void SctpAssociation::on_data(uint8_t flags, const uint8_t* v, size_t n) {
    if (n <= 12) return;  // empty DATA is a protocol violation; drop it
    const uint32_t tsn = rd32(v);
    if (le(tsn, peer_cum_)) {
        if (dups_.size() < 16) dups_.push_back(tsn);
        stats_.dup_tsns++;
        return;
    }
    const uint32_t off = tsn - peer_itsn_;
    if (above_.count(off)) {
        if (dups_.size() < 16) dups_.push_back(tsn);
        stats_.dup_tsns++;
        return;
    }
    const size_t len = n - 12;
    if (buffered_in_ + len > 4 * (size_t)kRwnd) return;  // out of buffer: the peer retransmits later
    InChunk c;
    c.stream = rd16(v + 4);
    c.ssn = rd16(v + 6);
    c.ppid = rd32(v + 8);
    c.flags = flags & 7;
    c.data.assign((const char*)v + 12, len);
    buffered_in_ += len;
    above_.insert(off);
    frags_.emplace(off, std::move(c));
    stats_.data_in++;
    advance_peer_cum();
    deliver_from(off);
}

void SctpAssociation::advance_peer_cum() {
    while (!above_.empty() && *above_.begin() == peer_cum_ + 1 - peer_itsn_) {
        above_.erase(above_.begin());
        ++peer_cum_;
    }
}

// Reassemble the message the chunk at TSN offset `off` belongs to, if all its fragments
// (consecutive TSNs from a B chunk to an E chunk, RFC 4960 6.9) are here.
void SctpAssociation::deliver_from(uint32_t off) {
    auto it = frags_.find(off);
    if (it == frags_.end()) return;
    const uint16_t stream = it->second.stream;
    uint32_t b = off;
    while (!(frags_.at(b).flags & F_B)) {
        auto p = frags_.find(b - 1);
        if (p == frags_.end() || p->second.stream != stream || (p->second.flags & F_E)) return;
        --b;
    }
    uint32_t e = off;
    while (!(frags_.at(e).flags & F_E)) {
        auto q = frags_.find(e + 1);
        if (q == frags_.end() || q->second.stream != stream || (q->second.flags & F_B)) return;
        ++e;
    }
    SctpMessage m;
    const InChunk& f = frags_.at(b);
    m.stream = f.stream;
    m.ppid = f.ppid;
    m.unordered = f.flags & F_U;
    const uint16_t ssn = f.ssn;
    for (uint32_t k = b;; ++k) {
        auto q = frags_.find(k);
        m.data += q->second.data;
        buffered_in_ -= q->second.data.size();
        frags_.erase(q);
        if (k == e) break;
    }
    stats_.messages_in++;
    if (m.unordered) {
        delivered_.push_back(std::move(m));
    } else {
        ordered_[stream].emplace(ssn, std::move(m));
        deliver_ordered(stream);
    }
}

void SctpAssociation::deliver_ordered(uint16_t stream) {
    auto& q = ordered_[stream];
    uint16_t& nx = in_ssn_[stream];
    for (auto it = q.find(nx); it != q.end(); it = q.find(nx)) {
        delivered_.push_back(std::move(it->second));
        q.erase(it);
        ++nx;
    }
}

void SctpAssociation::on_forward_tsn(const uint8_t* v, size_t n) {
    if (n < 4) return;
    stats_.forward_tsn_in++;
    const uint32_t ncum = rd32(v);
    if (le(ncum, peer_cum_)) return;
    const uint32_t lim = ncum - peer_itsn_;
    // drop every fragment the sender has abandoned (all TSNs up to the new cumulative point)
    for (auto it = frags_.begin(); it != frags_.end() && it->first <= lim;) {
        buffered_in_ -= it->second.data.size();
        it = frags_.erase(it);
    }
    while (!above_.empty() && *above_.begin() <= lim) above_.erase(above_.begin());
    peer_cum_ = ncum;
    advance_peer_cum();
    for (size_t o = 4; o + 4 <= n; o += 4) {  // skipped ordered messages: (stream, ssn)
        const uint16_t s = rd16(v + o), ssn = rd16(v + o + 2);
        uint16_t& nx = in_ssn_[s];
        if ((int16_t)(ssn - nx) >= 0) {
            auto& q = ordered_[s];
            for (auto it = q.begin(); it != q.end();)
                it = (int16_t)(it->first - ssn) <= 0 ? q.erase(it) : std::next(it);
            nx = (uint16_t)(ssn + 1);
        }
        deliver_ordered(s);
    }
    // a message whose later fragments arrived before the FORWARD-TSN may now be complete
    if (!frags_.empty()) deliver_from(frags_.begin()->first);
}

std::string SctpAssociation::make_sack() {
    std::string v;
    put32(v, peer_cum_);
    put32(v, kRwnd - (uint32_t)std::min<size_t>(buffered_in_, kRwnd));
    std::vector<std::pair<uint16_t, uint16_t>> gaps;
    const uint32_t base = peer_cum_ - peer_itsn_;  // offset of the cumulative point
    for (uint32_t off : above_) {
        const uint32_t rel = off - base;
        if (rel > 65535) break;
        if (!gaps.empty() && gaps.back().second + 1 == rel)
            gaps.back().second = (uint16_t)rel;
        else if (gaps.size() < 64)
            gaps.emplace_back((uint16_t)rel, (uint16_t)rel);
        else
            break;
    }
    put16(v, (uint16_t)gaps.size());
    put16(v, (uint16_t)dups_.size());
    for (auto& g : gaps) {
        put16(v, g.first);
        put16(v, g.second);
    }
    for (uint32_t d : dups_) put32(v, d);
    dups_.clear();
    stats_.sacks_out++;
    return chunk(C_SACK, 0, v);
}

// ---------------------------------------------------------------------- send side
std::vector<std::string> SctpAssociation::send(uint16_t stream, uint32_t ppid, const std::string& data,
                                               bool unordered, int max_retransmits, int lifetime_ms) {
    if (state_ != State::Closed && state_ != State::CookieWait && state_ != State::CookieEchoed &&
        state_ != State::Established)
        throw std::runtime_error("SCTP: association is shutting down or closed");
    if (data.empty()) throw std::invalid_argument("SCTP: empty user message");
    if (data.size() > max_message_) throw std::length_error("SCTP: message larger than max-message-size");
    const uint64_t msg = next_msg_++;
    const uint16_t ssn = unordered ? 0 : out_ssn_[stream]++;
    const int64_t expiry = lifetime_ms >= 0 ? now() + lifetime_ms : -1;
    for (size_t o = 0; o < data.size(); o += kMaxFragment) {
        OutChunk c;
        c.stream = stream;
        c.ssn = ssn;
        c.ppid = ppid;
        c.flags = (uint8_t)((unordered ? F_U : 0) | (o == 0 ? F_B : 0) | (o + kMaxFragment >= data.size() ? F_E : 0));
        c.data = data.substr(o, kMaxFragment);
        c.msg = msg;
        c.max_rtx = max_retransmits;
        c.expiry_ms = expiry;
        queue_.push_back(std::move(c));
    }
    stats_.messages_out++;
    return established() ? flush() : std::vector<std::string>{};
}

size_t SctpAssociation::buffered_amount() const {
    size_t n = 0;
    for (const auto& c : queue_) n += c.data.size();
    for (const auto& c : sent_)
        if (!c.acked && !c.abandoned) n += c.data.size();
    return n;
}

void SctpAssociation::on_sack(const uint8_t* v, size_t n) {
    if (n < 12) return;
    const uint32_t cum = rd32(v), rwnd = rd32(v + 4);
    const uint16_t ngap = rd16(v + 8);
    if (lt(cum, cum_acked_) || !lt(cum, next_tsn_)) return;  // stale, or acks what we never sent
    stats_.sacks_in++;
    const int64_t t = now();
    const bool advanced = lt(cum_acked_, cum);
    uint32_t acked_bytes = 0;
    bool sampled = false;
    auto ack_one = [&](OutChunk& c) {
        if (c.acked || c.abandoned) return;
        acked_bytes += (uint32_t)c.data.size();
        if (c.tx == 1 && !sampled) {  // Karn: only chunks sent once give an RTT sample
            const uint32_t r = (uint32_t)std::max<int64_t>(1, t - c.sent_ms);
            if (!have_rtt_) {
                srtt_ = r;
                rttvar_ = r / 2;
                have_rtt_ = true;
            } else {
                const uint32_t d = srtt_ > r ? srtt_ - r : r - srtt_;
                rttvar_ = (3 * rttvar_ + d) / 4;
                srtt_ = (7 * srtt_ + r) / 8;
            }
            rto_ = std::min(kRtoMax, std::max(kRtoMin, srtt_ + std::max(4 * rttvar_, 10u)));
            sampled = true;
        }
        c.acked = true;
    };
    while (!sent_.empty() && le(sent_.front().tsn, cum)) {
        ack_one(sent_.front());
        sent_.pop_front();
    }
    if (advanced) cum_acked_ = cum;
    if (lt(ack_point_, cum_acked_)) ack_point_ = cum_acked_;
    uint32_t highest = cum;
    for (size_t g = 0; g < ngap && 12 + 4 * g + 4 <= n; ++g) {
        const uint16_t s = rd16(v + 12 + 4 * g), e = rd16(v + 14 + 4 * g);
        for (uint32_t k = s; k <= e && s >= 1; ++k) {
            const uint32_t tsn = cum + k;
            if (sent_.empty() || lt(tsn, sent_.front().tsn)) continue;
            const size_t idx = tsn - sent_.front().tsn;
            if (idx >= sent_.size()) break;
            ack_one(sent_[idx]);
            if (lt(highest, tsn)) highest = tsn;
        }
    }
    // miss indications for chunks below the highest gap-acked TSN (RFC 4960 7.2.4)
    bool fast = false;
    for (auto& c : sent_) {
        if (!lt(c.tsn, highest)) break;
        if (c.acked || c.abandoned || c.rtx) continue;
        if (++c.miss == 3) {
            c.rtx = true;
            fast = true;
            stats_.fast_retransmits++;
        }
    }
    if (fast && !in_recovery_) {
        ssthresh_ = std::max(cwnd_ / 2, 4 * kMtu);
        cwnd_ = ssthresh_;
        partial_acked_ = 0;
        in_recovery_ = true;
        recover_tsn_ = next_tsn_ - 1;
    }
    if (in_recovery_ && le(recover_tsn_, cum_acked_)) in_recovery_ = false;
    if (advanced && !in_recovery_) {
        if (cwnd_ <= ssthresh_) {
            cwnd_ += std::min(acked_bytes, kMtu);
        } else {
            partial_acked_ += acked_bytes;
            if (partial_acked_ >= cwnd_) {
                partial_acked_ -= cwnd_;
                cwnd_ += kMtu;
            }
        }
    }
    uint32_t flight = 0;
    bool outstanding = false;
    for (const auto& c : sent_)
        if (!c.acked && !c.abandoned) {
            outstanding = true;
            if (!c.rtx) flight += (uint32_t)c.data.size();
        }
    peer_rwnd_ = rwnd > flight ? rwnd - flight : 0;
    if (advanced) {
        errors_ = 0;
        t3_deadline_ = outstanding ? t + rto_ : -1;
    } else if (!outstanding) {
        t3_deadline_ = -1;
    }
}

void SctpAssociation::abandon_message(uint64_t msg) {
    bool any = false;
    for (auto& c : sent_)
        if (c.msg == msg && !c.abandoned) {
            c.abandoned = true;
            c.rtx = false;
            any = true;
        }
    for (auto it = queue_.begin(); it != queue_.end();)
        if (it->msg == msg) {
            it = queue_.erase(it);
            any = true;
        } else {
            ++it;
        }
    if (any) stats_.abandoned++;
}

void SctpAssociation::on_t3_expiry() {
    stats_.t3_expiries++;
    rto_ = std::min(kRtoMax, rto_ * 2);
    ssthresh_ = std::max(cwnd_ / 2, 4 * kMtu);
    cwnd_ = kMtu;
    partial_acked_ = 0;
    in_recovery_ = false;
    for (auto& c : sent_)
        if (!c.acked && !c.abandoned) c.rtx = true;
    t3_deadline_ = -1;
    if (++errors_ > kMaxAssocRetrans) fail("association retransmission limit reached");
}

std::string SctpAssociation::make_reconfig_request() {
    std::string v;
    put32(v, reset_req_seq_);
    put32(v, peer_reconf_seq_ - 1);  // last request sequence number received from the peer
    put32(v, reset_last_tsn_);
    for (uint16_t s : reset_inflight_) put16(v, s);
    return chunk(C_RECONFIG, 0, param(P_OUT_RESET, v).substr(0, 4 + v.size()));
}

void SctpAssociation::on_reconfig(const uint8_t* v, size_t n, std::vector<std::string>& out) {
    (void)out;
    for (size_t o = 0; o + 4 <= n;) {
        const uint16_t pt = rd16(v + o), pl = rd16(v + o + 2);
        if (pl < 4 || o + pl > n) break;
        const uint8_t* pv = v + o + 4;
        const size_t plen = pl - 4;
        if (pt == P_OUT_RESET && plen >= 12) {
            const uint32_t req = rd32(pv), last_tsn = rd32(pv + 8);
            uint32_t result;
            if (last_reconf_valid_ && req == last_reconf_seq_ && last_reconf_result_ != 6) {
                result = last_reconf_result_;  // retransmitted request: repeat the answer
            } else if (le(last_tsn, peer_cum_)) {
                std::vector<uint16_t> streams;
                for (size_t k = 12; k + 2 <= plen; k += 2) streams.push_back(rd16(pv + k));
                if (streams.empty())
                    for (auto& kv : in_ssn_) streams.push_back(kv.first);
                for (uint16_t s : streams) {
                    in_ssn_[s] = 0;
                    ordered_.erase(s);
                    reset_in_.push_back(s);
                }
                result = 1;  // success, performed
            } else {
                result = 6;  // in progress: data up to last_tsn is still missing
            }
            last_reconf_valid_ = true;
            last_reconf_seq_ = req;
            last_reconf_result_ = result;
            if (!lt(req, peer_reconf_seq_)) peer_reconf_seq_ = req + 1;
            std::string r;
            put32(r, req);
            put32(r, result);
            ctrl_.push_back(chunk(C_RECONFIG, 0, param(P_RECONFIG_RESP, r)));
        } else if (pt == P_IN_RESET && plen >= 4) {
            std::string r;
            put32(r, rd32(pv));
            put32(r, 2);  // denied: we reset our outgoing streams ourselves
            ctrl_.push_back(chunk(C_RECONFIG, 0, param(P_RECONFIG_RESP, r)));
        } else if (pt == P_RECONFIG_RESP && plen >= 8) {
            const uint32_t seq = rd32(pv), result = rd32(pv + 4);
            if (!reset_inflight_.empty() && seq == reset_req_seq_) {
                if (result == 6) {
                    reconf_deadline_ = now() + rto_;  // ask again later
                } else {
                    if (result <= 1)
                        for (uint16_t s : reset_inflight_) out_ssn_[s] = 0;
                    reset_inflight_.clear();
                    reconf_deadline_ = -1;
                }
            }
        }
        o += pad4(pl);
    }
}

// Gather control chunks, SACK, FORWARD-TSN, retransmissions and new DATA (within cwnd and
// the peer's window) into packets of at most kMaxPacket bytes.
std::vector<std::string> SctpAssociation::flush() {
    std::vector<std::string> chunks;
    for (auto& c : ctrl_) chunks.push_back(std::move(c));
    ctrl_.clear();
    if (sack_pending_) {
        chunks.push_back(make_sack());
        sack_pending_ = false;
    }
    const bool can_send = state_ == State::Established || state_ == State::ShutdownPending ||
                          state_ == State::ShutdownReceived;
    if (can_send) {
        const int64_t t = now();
        // partial reliability: abandon what is over its retransmission or lifetime budget
        for (auto& c : sent_) {
            if (c.acked || c.abandoned) continue;
            if ((c.rtx && c.max_rtx >= 0 && c.tx > c.max_rtx) || (c.expiry_ms >= 0 && t >= c.expiry_ms && c.rtx))
                abandon_message(c.msg);
        }
        ack_point_ = cum_acked_;
        for (const auto& c : sent_) {
            if (!c.abandoned) break;
            ack_point_ = c.tsn;
        }
        if (lt(cum_acked_, ack_point_) && peer_prsctp_) {
            std::string v;
            put32(v, ack_point_);
            std::map<uint16_t, uint16_t> skip;
            for (const auto& c : sent_) {
                if (lt(ack_point_, c.tsn)) break;
                if (!(c.flags & F_U)) skip[c.stream] = c.ssn;
            }
            for (auto& kv : skip) {
                put16(v, kv.first);
                put16(v, kv.second);
            }
            chunks.push_back(chunk(C_FORWARD_TSN, 0, v));
            stats_.forward_tsn_out++;
            if (t3_deadline_ < 0) t3_deadline_ = t + rto_;
        }
        uint32_t flight = 0;
        for (const auto& c : sent_)
            if (!c.acked && !c.abandoned && !c.rtx) flight += (uint32_t)c.data.size();
        auto data_chunk = [&](const OutChunk& c) {
            std::string v;
            v.reserve(12 + c.data.size());
            put32(v, c.tsn);
            put16(v, c.stream);
            put16(v, c.ssn);
            put32(v, c.ppid);
            v += c.data;
            return chunk(C_DATA, c.flags, v);
        };
        bool sent_data = false;
        for (auto& c : sent_) {  // retransmissions first, one packet's worth even when cwnd is full
            if (!c.rtx || c.acked || c.abandoned) continue;
            if (sent_data && flight + c.data.size() > cwnd_) break;
            chunks.push_back(data_chunk(c));
            c.rtx = false;
            c.miss = 0;
            c.tx++;
            c.sent_ms = t;
            flight += (uint32_t)c.data.size();
            stats_.retransmits++;
            sent_data = true;
        }
        while (!queue_.empty()) {
            OutChunk& c = queue_.front();
            if (c.expiry_ms >= 0 && t >= c.expiry_ms && (c.flags & F_B)) {  // expired before it left
                abandon_message(c.msg);
                continue;
            }
            const uint32_t sz = (uint32_t)c.data.size();
            if (flight > 0 && (flight + sz > cwnd_ || sz > peer_rwnd_)) break;
            c.tsn = next_tsn_++;
            c.tx = 1;
            c.sent_ms = t;
            chunks.push_back(data_chunk(c));
            peer_rwnd_ -= std::min(sz, peer_rwnd_);
            flight += sz;
            sent_.push_back(std::move(c));
            queue_.pop_front();
            stats_.data_out++;
            sent_data = true;
        }
        if (sent_data && t3_deadline_ < 0) t3_deadline_ = t + rto_;
        // stream reset once everything queued on those streams has a TSN
        if (reset_inflight_.empty() && !reset_pending_.empty()) {
            bool busy = false;
            for (const auto& c : queue_)
                busy |= std::find(reset_pending_.begin(), reset_pending_.end(), c.stream) != reset_pending_.end();
            if (!busy) {
                reset_inflight_.swap(reset_pending_);
                reset_req_seq_ = my_reconf_seq_++;
                reset_last_tsn_ = next_tsn_ - 1;
                chunks.push_back(make_reconfig_request());
                reconf_deadline_ = t + rto_;
            }
        }
        bool idle = queue_.empty();
        for (const auto& c : sent_) idle &= c.acked || c.abandoned;
        if (idle && state_ == State::ShutdownPending) {
            std::string v;
            put32(v, peer_cum_);
            chunks.push_back(chunk(C_SHUTDOWN, 0, v));
            state_ = State::ShutdownSent;
            t2_deadline_ = t + rto_;
        } else if (idle && state_ == State::ShutdownReceived) {
            chunks.push_back(chunk(C_SHUTDOWN_ACK, 0, ""));
            state_ = State::ShutdownAckSent;
            t2_deadline_ = t + rto_;
        }
    }
    std::vector<std::string> out;
    std::vector<std::string> cur;
    size_t cur_len = 12;
    for (auto& c : chunks) {
        const size_t l = pad4(c.size());
        if (!cur.empty() && cur_len + l > kMaxPacket) {
            out.push_back(build(cur, peer_tag_));
            cur.clear();
            cur_len = 12;
        }
        cur_len += l;
        cur.push_back(std::move(c));
    }
    if (!cur.empty()) out.push_back(build(cur, peer_tag_));
    stats_.packets_out += out.size();
    return out;
}

std::vector<std::string> SctpAssociation::tick() {
    std::vector<std::string> out;
    const int64_t t = now();
    if (t1_deadline_ >= 0 && t >= t1_deadline_) {
        if (++t1_tries_ > kMaxInitRetrans) {
            fail("association setup timed out");
            return out;
        }
        rto_ = std::min(kRtoMax, rto_ * 2);
        t1_deadline_ = t + rto_;
        if (state_ == State::CookieWait)
            out.push_back(build({make_init_chunk(C_INIT, my_tag_, my_itsn_, "")}, 0));
        else if (state_ == State::CookieEchoed)
            out.push_back(build({chunk(C_COOKIE_ECHO, 0, cookie_)}, peer_tag_));
        stats_.packets_out += out.size();
        return out;
    }
    if (t3_deadline_ >= 0 && t >= t3_deadline_) {
        on_t3_expiry();
        if (state_ == State::Aborted) {
            out.push_back(build({chunk(C_ABORT, 0, "")}, peer_tag_));
            return out;
        }
    }
    if (reconf_deadline_ >= 0 && t >= reconf_deadline_ && !reset_inflight_.empty()) {
        ctrl_.push_back(make_reconfig_request());
        reconf_deadline_ = t + rto_;
    }
    if (t2_deadline_ >= 0 && t >= t2_deadline_) {
        if (state_ == State::ShutdownSent) {
            std::string v;
            put32(v, peer_cum_);
            ctrl_.push_back(chunk(C_SHUTDOWN, 0, v));
        } else if (state_ == State::ShutdownAckSent) {
            ctrl_.push_back(chunk(C_SHUTDOWN_ACK, 0, ""));
        }
        rto_ = std::min(kRtoMax, rto_ * 2);
        t2_deadline_ = t + rto_;
    }
    for (auto& s : flush()) out.push_back(std::move(s));
    return out;
}

std::vector<std::string> SctpAssociation::reset_streams(const std::vector<uint16_t>& streams) {
    if (!established()) return {};
    for (uint16_t s : streams)
        if (std::find(reset_pending_.begin(), reset_pending_.end(), s) == reset_pending_.end())
            reset_pending_.push_back(s);
    return flush();
}

std::vector<std::string> SctpAssociation::shutdown() {
    if (state_ == State::Established) {
        state_ = State::ShutdownPending;
        return flush();
    }
    if (state_ == State::CookieWait || state_ == State::CookieEchoed) {
        state_ = State::Closed;
        t1_deadline_ = -1;
    }
    return {};
}

std::vector<std::string> SctpAssociation::abort(const std::string& reason) {
    if (state_ == State::Closed || state_ == State::Aborted) return {};
    std::string cause;
    put16(cause, 12);  // user-initiated abort
    put16(cause, (uint16_t)(4 + reason.size()));
    cause += reason;
    const uint32_t tag = peer_tag_;
    fail("aborted: " + reason);
    std::vector<std::string> out{build({chunk(C_ABORT, 0, cause)}, tag)};
    stats_.packets_out++;
    return out;
}

std::vector<SctpMessage> SctpAssociation::take_messages() {
    std::vector<SctpMessage> m;
    m.swap(delivered_);
    return m;
}

std::vector<uint16_t> SctpAssociation::take_reset_streams() {
    std::vector<uint16_t> r;
    r.swap(reset_in_);
    return r;
}

// ====================================================================== data channels
namespace {
enum : uint32_t { PPID_DCEP = 50, PPID_STRING = 51, PPID_BINARY = 53, PPID_STRING_EMPTY = 56, PPID_BINARY_EMPTY = 57 };
enum : uint8_t { DCEP_ACK = 0x02, DCEP_OPEN = 0x03 };
enum : uint8_t { CH_RELIABLE = 0x00, CH_REXMIT = 0x01, CH_TIMED = 0x02, CH_UNORDERED = 0x80 };
}  // namespace

DataChannelEndpoint::DataChannelEndpoint(bool dtls_server, uint16_t local_port, uint16_t remote_port,
                                         size_t max_message)
    : sctp_(local_port, remote_port, max_message), next_id_(dtls_server ? 1 : 0) {}

std::vector<std::string> DataChannelEndpoint::feed(const std::string& packet) {
    std::vector<std::string> out = sctp_.feed(packet);
    process();
    for (auto& p : out_) out.push_back(std::move(p));
    out_.clear();
    return out;
}

void DataChannelEndpoint::process() {
    auto emit = [&](std::vector<std::string> v) {
        for (auto& p : v) out_.push_back(std::move(p));
    };
    for (auto& m : sctp_.take_messages()) {
        if (m.ppid == PPID_DCEP) {
            const uint8_t* d = (const uint8_t*)m.data.data();
            if (!m.data.empty() && d[0] == DCEP_OPEN && m.data.size() >= 12) {
                const uint8_t type = d[1];
                const uint32_t rel = rd32(d + 4);
                const size_t ll = rd16(d + 8), pl = rd16(d + 10);
                if (12 + ll + pl > m.data.size()) continue;
                Channel c;
                c.label = m.data.substr(12, ll);
                c.protocol = m.data.substr(12 + ll, pl);
                c.ordered = !(type & CH_UNORDERED);
                c.max_rtx = (type & 0x7f) == CH_REXMIT ? (int)rel : -1;
                c.lifetime = (type & 0x7f) == CH_TIMED ? (int)rel : -1;
                c.acked = true;
                ch_[m.stream] = c;
                emit(sctp_.send(m.stream, PPID_DCEP, std::string(1, (char)DCEP_ACK)));
                DataChannelEvent e;
                e.kind = DataChannelEvent::Open;
                e.id = m.stream;
                e.label = c.label;
                e.protocol = c.protocol;
                events_.push_back(std::move(e));
            } else if (!m.data.empty() && d[0] == DCEP_ACK) {
                auto it = ch_.find(m.stream);
                if (it != ch_.end() && !it->second.acked) {
                    it->second.acked = true;
                    DataChannelEvent e;
                    e.kind = DataChannelEvent::Open;
                    e.id = m.stream;
                    e.label = it->second.label;
                    e.protocol = it->second.protocol;
                    events_.push_back(std::move(e));
                }
            }
            continue;
        }
        auto it = ch_.find(m.stream);
        if (it == ch_.end()) continue;
        DataChannelEvent e;
        e.kind = DataChannelEvent::Message;
        e.id = m.stream;
        e.binary = m.ppid == PPID_BINARY || m.ppid == PPID_BINARY_EMPTY || m.ppid == 52;
        if (m.ppid != PPID_STRING_EMPTY && m.ppid != PPID_BINARY_EMPTY) e.data = std::move(m.data);
        events_.push_back(std::move(e));
    }
    for (uint16_t s : sctp_.take_reset_streams()) {
        auto it = ch_.find(s);
        if (it == ch_.end()) continue;
        if (!it->second.closing) emit(sctp_.reset_streams({s}));  // close our direction too
        DataChannelEvent e;
        e.kind = DataChannelEvent::Closed;
        e.id = s;
        e.label = it->second.label;
        events_.push_back(std::move(e));
        ch_.erase(it);
    }
}

std::pair<int, std::vector<std::string>> DataChannelEndpoint::open(const std::string& label,
                                                                   const std::string& protocol, bool ordered,
                                                                   int max_retransmits, int max_lifetime_ms) {
    while (ch_.count(next_id_)) next_id_ = (uint16_t)(next_id_ + 2);
    const uint16_t id = next_id_;
    next_id_ = (uint16_t)(next_id_ + 2);
    uint8_t type = ordered ? 0 : CH_UNORDERED;
    uint32_t rel = 0;
    if (max_retransmits >= 0) {
        type |= CH_REXMIT;
        rel = (uint32_t)max_retransmits;
    } else if (max_lifetime_ms >= 0) {
        type |= CH_TIMED;
        rel = (uint32_t)max_lifetime_ms;
    }
    std::string m;
    put8(m, DCEP_OPEN);
    put8(m, type);
    put16(m, 0);  // priority
    put32(m, rel);
    put16(m, (uint16_t)label.size());
    put16(m, (uint16_t)protocol.size());
    m += label;
    m += protocol;
    Channel c;
    c.label = label;
    c.protocol = protocol;
    c.ordered = ordered;
    c.max_rtx = max_retransmits;
    c.lifetime = max_retransmits >= 0 ? -1 : max_lifetime_ms;
    ch_[id] = c;
    return {id, sctp_.send(id, PPID_DCEP, m)};
}

std::vector<std::string> DataChannelEndpoint::send(uint16_t id, const std::string& data, bool binary) {
    auto it = ch_.find(id);
    if (it == ch_.end() || it->second.closing) throw std::runtime_error("data channel is not open");
    const Channel& c = it->second;
    const uint32_t ppid = binary ? (data.empty() ? PPID_BINARY_EMPTY : PPID_BINARY)
                                 : (data.empty() ? PPID_STRING_EMPTY : PPID_STRING);
    // until the peer has acknowledged the OPEN, messages stay ordered (RFC 8832 6)
    return sctp_.send(id, ppid, data.empty() ? std::string(1, '\0') : data, !c.ordered && c.acked, c.max_rtx,
                      c.lifetime);
}

std::vector<std::string> DataChannelEndpoint::close(uint16_t id) {
    auto it = ch_.find(id);
    if (it == ch_.end() || it->second.closing) return {};
    it->second.closing = true;
    return sctp_.reset_streams({id});
}

std::vector<DataChannelEvent> DataChannelEndpoint::take_events() {
    std::vector<DataChannelEvent> e;
    e.swap(events_);
    return e;
}

bool DataChannelEndpoint::is_open(uint16_t id) const {
    auto it = ch_.find(id);
    return it != ch_.end() && it->second.acked && !it->second.closing;
}

std::string DataChannelEndpoint::label(uint16_t id) const {
    auto it = ch_.find(id);
    return it == ch_.end() ? std::string() : it->second.label;
}

std::vector<uint16_t> DataChannelEndpoint::channels() const {
    std::vector<uint16_t> v;
    for (auto& kv : ch_) v.push_back(kv.first);
    return v;
}

}  // namespace net
}  // namespace mx
