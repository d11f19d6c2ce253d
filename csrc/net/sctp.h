// SCTP over DTLS (RFC 8261) and WebRTC data channels (RFC 8831 / DCEP RFC 8832).
//
// The reference gets its data channels from GStreamer webrtcbin + usrsctp; selkies carries
// keyboard / mouse / clipboard / gamepad input and stats on a channel named "input"
// (SURVEY.md C37, C52).  This is a native user-space SCTP engine sized for that job:
//
//   * SctpAssociation -- one association, driven through memory (feed a received SCTP
//     packet, get packets to send; the caller wraps them in DTLS records).  Four-way
//     handshake with an HMAC-signed state cookie (RFC 4960 5.1), DATA fragmentation and
//     reassembly, ordered / unordered delivery, SACK with gap blocks and duplicate
//     reports, RTO estimation (RFC 6298 constants, 200 ms floor), T1/T3 timers with
//     backoff, fast retransmit after three miss indications, slow start / congestion
//     avoidance, partial reliability (RFC 3758 FORWARD-TSN, limited retransmissions and
//     lifetimes), stream reset (RFC 6525 outgoing SSN reset request / response),
//     HEARTBEAT echo, ABORT and graceful SHUTDOWN.
//   * DataChannelEndpoint -- DCEP open / ack, string / binary / empty PPIDs, channel
//     close by stream reset, stream-id parity by DTLS role (client even, server odd).
//
// Not implemented (not used by browsers' data channels): multi-homing, I-DATA
// interleaving (RFC 8260), ASCONF, AUTH chunks.
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace mx {
namespace net {

// CRC-32C (Castagnoli, reflected polynomial 0x82F63B78) -- the SCTP checksum (RFC 4960 App. B).
uint32_t crc32c(const void* data, size_t n);

struct SctpMessage {
    uint16_t stream = 0;
    uint32_t ppid = 0;
    bool unordered = false;
    std::string data;
};

struct SctpStats {
    uint64_t packets_in = 0, packets_out = 0;
    uint64_t data_in = 0, data_out = 0;  // DATA chunks (first transmissions)
    uint64_t retransmits = 0, fast_retransmits = 0, t3_expiries = 0;
    uint64_t abandoned = 0, forward_tsn_out = 0, forward_tsn_in = 0;
    uint64_t sacks_in = 0, sacks_out = 0, dup_tsns = 0;
    uint64_t bad_checksum = 0, bad_tag = 0;
    uint64_t messages_in = 0, messages_out = 0;
};

class SctpAssociation {
   public:
    enum class State { Closed, CookieWait, CookieEchoed, Established, ShutdownPending, ShutdownSent,
                       ShutdownReceived, ShutdownAckSent, Aborted };
    static constexpr size_t kMaxPacket = 1100;  // SCTP packet incl. common header (fits one DTLS record < 1200)
    static constexpr size_t kDataHeader = 16;
    static constexpr size_t kMaxFragment = kMaxPacket - 12 - kDataHeader;
    static constexpr uint32_t kRwnd = 1u << 20;

    explicit SctpAssociation(uint16_t local_port = 5000, uint16_t remote_port = 5000,
                             size_t max_message = 256 * 1024);

    // Active open (sends INIT).  The passive side never calls this: it answers INIT.
    std::vector<std::string> connect();
    // One received SCTP packet (the payload of a DTLS application-data record).
    std::vector<std::string> feed(const std::string& packet);
    // Queue one user message; returns what the windows allow to go out now.  Messages
    // queued before the association is established go out once it is.
    // max_retransmits / lifetime_ms < 0: fully reliable.
    std::vector<std::string> send(uint16_t stream, uint32_t ppid, const std::string& data, bool unordered = false,
                                  int max_retransmits = -1, int lifetime_ms = -1);
    // Timers (T1-init/cookie, T3-rtx, reconfig, T2-shutdown); call every few tens of ms.
    std::vector<std::string> tick();
    // RFC 6525 outgoing SSN reset of our streams (how a data channel is closed).
    std::vector<std::string> reset_streams(const std::vector<uint16_t>& streams);
    std::vector<std::string> shutdown();
    std::vector<std::string> abort(const std::string& reason);

    std::vector<SctpMessage> take_messages();
    std::vector<uint16_t> take_reset_streams();  // incoming streams the peer has reset

    State state() const { return state_; }
    bool established() const { return state_ == State::Established; }
    const SctpStats& stats() const { return stats_; }
    size_t buffered_amount() const;  // queued + unacknowledged user bytes
    uint32_t rto_ms() const { return rto_; }
    uint32_t cwnd() const { return cwnd_; }
    uint32_t peer_rwnd() const { return peer_rwnd_; }
    bool peer_supports_forward_tsn() const { return peer_prsctp_; }
    std::string error() const { return err_; }
    // Tests: pin the clock (ms); a negative value restores the steady clock.
    void set_clock(int64_t ms) { clock_ = ms; }

   private:
    struct OutChunk {
        uint32_t tsn = 0;
        uint16_t stream = 0, ssn = 0;
        uint32_t ppid = 0;
        uint8_t flags = 0;  // U B E
        std::string data;
        uint64_t msg = 0;      // message serial (abandonment is per message)
        int64_t sent_ms = 0;
        int tx = 0;            // transmissions so far
        int miss = 0;          // fast-retransmit miss indications
        int max_rtx = -1;
        int64_t expiry_ms = -1;
        bool acked = false;    // gap-acked
        bool abandoned = false;
        bool rtx = false;      // marked for retransmission
    };
    struct InChunk {
        uint16_t stream = 0, ssn = 0;
        uint32_t ppid = 0;
        uint8_t flags = 0;
        std::string data;
    };

    int64_t now() const;
    std::string build(const std::vector<std::string>& chunks, uint32_t vtag) const;
    std::vector<std::string> flush();
    void on_chunk(uint8_t type, uint8_t flags, const uint8_t* v, size_t n, std::vector<std::string>& out,
                  bool& sack_needed, bool& stop);
    void on_init(const uint8_t* v, size_t n, bool ack, std::vector<std::string>& out);
    void on_cookie_echo(const uint8_t* v, size_t n, std::vector<std::string>& out);
    void on_data(uint8_t flags, const uint8_t* v, size_t n);
    void on_sack(const uint8_t* v, size_t n);
    void on_forward_tsn(const uint8_t* v, size_t n);
    void on_reconfig(const uint8_t* v, size_t n, std::vector<std::string>& out);
    void deliver_from(uint32_t off);
    void deliver_ordered(uint16_t stream);
    void advance_peer_cum();
    std::string make_sack();
    std::string make_init_chunk(uint8_t type, uint32_t tag, uint32_t itsn, const std::string& cookie) const;
    std::string make_reconfig_request();
    std::string make_cookie(uint32_t peer_tag, uint32_t peer_itsn, uint32_t peer_rwnd, uint32_t my_tag,
                            uint32_t my_itsn, uint8_t ext) const;
    void abandon_message(uint64_t msg);
    void on_t3_expiry();
    void enter_established();
    void fail(const std::string& why);

    uint16_t lport_, rport_;
    size_t max_message_;
    State state_ = State::Closed;
    std::string err_;
    int64_t clock_ = -1;
    uint8_t secret_[32];

    // association
    uint32_t my_tag_ = 0, peer_tag_ = 0;
    uint32_t my_itsn_ = 0, peer_itsn_ = 0;
    bool peer_prsctp_ = false, peer_reconfig_ = false;
    std::string cookie_;  // (active side) cookie to echo
    uint32_t cur_vtag_ = 0;  // verification tag of the packet being processed
    bool sack_pending_ = false;
    std::vector<std::string> ctrl_;  // control chunks for the next packet
    int64_t t1_deadline_ = -1;
    int t1_tries_ = 0;

    // send side
    uint32_t next_tsn_ = 0;
    uint32_t cum_acked_ = 0;  // peer's cumulative ack of our TSNs
    uint32_t ack_point_ = 0;  // advanced peer ack point (RFC 3758)
    uint64_t next_msg_ = 1;
    std::map<uint16_t, uint16_t> out_ssn_;
    std::deque<OutChunk> queue_;  // not yet transmitted (no TSN)
    std::deque<OutChunk> sent_;   // TSN order, everything above cum_acked_
    uint32_t cwnd_ = 4380, ssthresh_ = kRwnd, partial_acked_ = 0, peer_rwnd_ = kRwnd;
    uint32_t rto_ = 1000, srtt_ = 0, rttvar_ = 0;
    bool have_rtt_ = false;
    int64_t t3_deadline_ = -1;
    int errors_ = 0;
    bool in_recovery_ = false;
    uint32_t recover_tsn_ = 0;

    // receive side
    uint32_t peer_cum_ = 0;         // last in-sequence TSN received
    std::set<uint32_t> above_;      // TSN offsets (from peer_itsn_) received above peer_cum_
    std::map<uint32_t, InChunk> frags_;  // undelivered chunks by TSN offset
    std::map<uint16_t, uint16_t> in_ssn_;  // next expected SSN per stream
    std::map<uint16_t, std::map<uint16_t, SctpMessage>> ordered_;  // complete but out of order
    std::vector<uint32_t> dups_;
    size_t buffered_in_ = 0;
    std::vector<SctpMessage> delivered_;

    // stream reset (RFC 6525)
    uint32_t my_reconf_seq_ = 0, peer_reconf_seq_ = 0;
    std::vector<uint16_t> reset_pending_;   // streams to reset, not yet requested
    std::vector<uint16_t> reset_inflight_;  // requested, awaiting response
    uint32_t reset_req_seq_ = 0, reset_last_tsn_ = 0;
    int64_t reconf_deadline_ = -1;
    std::vector<uint16_t> reset_in_;        // peer-reset incoming streams for the app
    bool last_reconf_valid_ = false;
    uint32_t last_reconf_seq_ = 0, last_reconf_result_ = 0;

    // shutdown
    int64_t t2_deadline_ = -1;

    SctpStats stats_;
};

// WebRTC data channels on top of one association (RFC 8831 / 8832).
struct DataChannelEvent {
    enum Kind { Open = 0, Message = 1, Closed = 2 };
    int kind = Open;
    uint16_t id = 0;
    std::string label, protocol;
    bool binary = false;
    std::string data;
};

class DataChannelEndpoint {
   public:
    // dtls_server: our DTLS role (server -> odd stream ids, client -> even).
    explicit DataChannelEndpoint(bool dtls_server, uint16_t local_port = 5000, uint16_t remote_port = 5000,
                                 size_t max_message = 256 * 1024);
    std::vector<std::string> connect() { return sctp_.connect(); }
    std::vector<std::string> feed(const std::string& packet);
    std::vector<std::string> tick() { return sctp_.tick(); }
    // Open a channel (DCEP DATA_CHANNEL_OPEN); returns its stream id and the packets to send.
    std::pair<int, std::vector<std::string>> open(const std::string& label, const std::string& protocol = "",
                                                  bool ordered = true, int max_retransmits = -1,
                                                  int max_lifetime_ms = -1);
    std::vector<std::string> send(uint16_t id, const std::string& data, bool binary);
    std::vector<std::string> close(uint16_t id);
    std::vector<DataChannelEvent> take_events();
    bool is_open(uint16_t id) const;
    std::string label(uint16_t id) const;
    std::vector<uint16_t> channels() const;
    SctpAssociation& sctp() { return sctp_; }

   private:
    struct Channel {
        std::string label, protocol;
        bool ordered = true;
        int max_rtx = -1, lifetime = -1;
        bool acked = false;  // peer has answered our OPEN (or we answered theirs)
        bool closing = false;
    };
    void process();

    SctpAssociation sctp_;
    uint16_t next_id_;
    std::map<uint16_t, Channel> ch_;
    std::vector<DataChannelEvent> events_;
    std::vector<std::string> out_;
};

}  // namespace net
}  // namespace mx
