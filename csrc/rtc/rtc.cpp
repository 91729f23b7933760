// Native WebRTC transport core: DTLS-SRTP handshake (OpenSSL, datagram BIO
// over in-process queues), SRTP/SRTCP AES_CM_128_HMAC_SHA1_80, RFC 6184 H.264
// packetisation and CRC32c. See rtc_api.h for the contract and the reference
// components it replaces (aiortc rtcdtlstransport.py / rtcrtpsender.py /
// codecs/h264.py, webrtcbin in legacy/gstwebrtc_app.py).
#include "rtc_api.h"

#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>
#include <openssl/srtp.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <string.h>

#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

using Bytes = std::vector<uint8_t>;

// ---------------------------------------------------------------------------
// DTLS
struct Dtls {
    SSL_CTX* ctx = nullptr;
    SSL* ssl = nullptr;
    EVP_PKEY* key = nullptr;
    X509* cert = nullptr;
    std::deque<Bytes> in, out, app;
    std::string local_fp, remote_fp, err;
    int role = 1;
    int state = 0;
};

BIO_METHOD* g_bio_method = nullptr;

int bio_write(BIO* b, const char* data, int len) {
    auto* d = static_cast<Dtls*>(BIO_get_data(b));
    d->out.emplace_back(reinterpret_cast<const uint8_t*>(data), reinterpret_cast<const uint8_t*>(data) + len);
    return len;
}

int bio_read(BIO* b, char* buf, int len) {
    auto* d = static_cast<Dtls*>(BIO_get_data(b));
    BIO_clear_retry_flags(b);
    if (d->in.empty()) {
        BIO_set_retry_read(b);
        return -1;
    }
    Bytes pkt = std::move(d->in.front());
    d->in.pop_front();
    int n = (int)pkt.size() < len ? (int)pkt.size() : len;  // datagram semantics: excess is dropped
    memcpy(buf, pkt.data(), n);
    return n;
}

long bio_ctrl(BIO* b, int cmd, long, void*) {
    auto* d = static_cast<Dtls*>(BIO_get_data(b));
    switch (cmd) {
        case BIO_CTRL_FLUSH: return 1;
        case BIO_CTRL_PENDING: return d->in.empty() ? 0 : (long)d->in.front().size();
        case BIO_CTRL_WPENDING: return 0;
        case BIO_CTRL_DGRAM_QUERY_MTU:
        case BIO_CTRL_DGRAM_GET_FALLBACK_MTU: return 1200;
        case BIO_CTRL_DGRAM_GET_MTU_OVERHEAD: return 28;  // IPv4 + UDP
        default: return 0;
    }
}

int bio_create(BIO* b) {
    BIO_set_init(b, 1);
    return 1;
}

BIO_METHOD* bio_method() {
    if (!g_bio_method) {
        g_bio_method = BIO_meth_new(BIO_get_new_index() | BIO_TYPE_SOURCE_SINK, "selkies-dgram");
        BIO_meth_set_write(g_bio_method, bio_write);
        BIO_meth_set_read(g_bio_method, bio_read);
        BIO_meth_set_ctrl(g_bio_method, bio_ctrl);
        BIO_meth_set_create(g_bio_method, bio_create);
    }
    return g_bio_method;
}

int verify_any(int, X509_STORE_CTX*) { return 1; }  // self-signed; the SDP fingerprint is the trust anchor

std::string fingerprint_of(X509* x) {
    unsigned char md[EVP_MAX_MD_SIZE];
    unsigned int n = 0;
    X509_digest(x, EVP_sha256(), md, &n);
    static const char* hex = "0123456789ABCDEF";
    std::string s;
    for (unsigned i = 0; i < n; i++) {
        if (i) s += ':';
        s += hex[md[i] >> 4];
        s += hex[md[i] & 15];
    }
    return s;
}

std::string upper(std::string s) {
    for (auto& c : s) c = (char)toupper((unsigned char)c);
    return s;
}

std::string ssl_errors() {
    std::string s;
    unsigned long e;
    char buf[256];
    while ((e = ERR_get_error()) != 0) {
        ERR_error_string_n(e, buf, sizeof buf);
        if (!s.empty()) s += "; ";
        s += buf;
    }
    return s;
}

bool make_identity(Dtls* d) {
    d->key = EVP_PKEY_Q_keygen(nullptr, nullptr, "EC", "P-256");
    if (!d->key) return false;
    d->cert = X509_new();
    X509_set_version(d->cert, 2);
    uint32_t serial = 0;
    RAND_bytes(reinterpret_cast<unsigned char*>(&serial), sizeof serial);
    ASN1_INTEGER_set(X509_get_serialNumber(d->cert), serial & 0x7fffffff);
    X509_gmtime_adj(X509_getm_notBefore(d->cert), -86400);
    X509_gmtime_adj(X509_getm_notAfter(d->cert), 30L * 86400);
    X509_set_pubkey(d->cert, d->key);
    X509_NAME* nm = X509_get_subject_name(d->cert);
    X509_NAME_add_entry_by_txt(nm, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("selkies"), -1, -1, 0);
    X509_set_issuer_name(d->cert, nm);
    if (!X509_sign(d->cert, d->key, EVP_sha256())) return false;
    d->local_fp = fingerprint_of(d->cert);
    return true;
}

int handshake_step(Dtls* d) {
    int r = SSL_do_handshake(d->ssl);
    if (r == 1) {
        X509* peer = SSL_get1_peer_certificate(d->ssl);
        if (!peer) {
            d->err = "peer sent no certificate";
            d->state = 3;
            return -1;
        }
        std::string fp = fingerprint_of(peer);
        X509_free(peer);
        if (!d->remote_fp.empty() && upper(d->remote_fp) != fp) {
            d->err = "remote fingerprint mismatch";
            d->state = 3;
            return -1;
        }
        const SRTP_PROTECTION_PROFILE* prof = SSL_get_selected_srtp_profile(d->ssl);
        if (!prof || prof->id != SRTP_AES128_CM_SHA1_80) {
            d->err = "no SRTP_AES128_CM_SHA1_80 profile negotiated";
            d->state = 3;
            return -1;
        }
        d->state = 2;
        return 1;
    }
    int e = SSL_get_error(d->ssl, r);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return 0;
    d->err = "handshake failed: " + ssl_errors();
    d->state = 3;
    return -1;
}

void drain_app(Dtls* d) {
    uint8_t buf[16384];
    for (;;) {
        int r = SSL_read(d->ssl, buf, sizeof buf);
        if (r > 0) {
            d->app.emplace_back(buf, buf + r);
            continue;
        }
        int e = SSL_get_error(d->ssl, r);
        if (e == SSL_ERROR_ZERO_RETURN) d->state = 4;
        else if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) ERR_clear_error();
        return;
    }
}

// ---------------------------------------------------------------------------
// SRTP (RFC 3711), AES_CM_128_HMAC_SHA1_80
struct Keys {
    uint8_t enc[16], salt[14], auth[20];
};

struct RecvState {
    bool init = false;
    uint32_t roc = 0;
    uint16_t s_l = 0;
    uint64_t max_index = 0;
    uint64_t window = 0;  // bit i: index max_index - i seen
};

struct Srtp {
    Keys rtp, rtcp;
    EVP_CIPHER_CTX* aes = nullptr;
    HMAC_CTX* hm_rtp = nullptr;
    HMAC_CTX* hm_rtcp = nullptr;
    std::unordered_map<uint32_t, std::pair<uint32_t, int>> send_roc;  // ssrc -> (roc, last seq or -1)
    std::unordered_map<uint32_t, uint32_t> send_rtcp_index;
    std::unordered_map<uint32_t, RecvState> recv;
    std::unordered_map<uint32_t, RecvState> recv_rtcp;
};

void aes_cm(EVP_CIPHER_CTX* c, const uint8_t* key, const uint8_t* iv, uint8_t* data, int n) {
    int outl = 0;
    EVP_EncryptInit_ex(c, EVP_aes_128_ctr(), nullptr, key, iv);
    EVP_EncryptUpdate(c, data, &outl, data, n);
}

void derive(EVP_CIPHER_CTX* c, const uint8_t* mkey, const uint8_t* msalt, int label, uint8_t* out, int n) {
    uint8_t iv[16] = {0};
    memcpy(iv, msalt, 14);
    iv[7] ^= (uint8_t)label;  // key_id = label || r (r = 0, kdr = 0), right-aligned against the salt
    memset(out, 0, n);
    aes_cm(c, mkey, iv, out, n);
}

void packet_iv(const uint8_t* salt, uint32_t ssrc, uint64_t index, uint8_t* iv) {
    memcpy(iv, salt, 14);
    iv[14] = iv[15] = 0;
    for (int i = 0; i < 4; i++) iv[4 + i] ^= (uint8_t)(ssrc >> (24 - 8 * i));
    for (int i = 0; i < 6; i++) iv[8 + i] ^= (uint8_t)(index >> (40 - 8 * i));
}

void tag(HMAC_CTX* h, const uint8_t* data, int n, const uint8_t* extra4, uint8_t* out10) {
    unsigned char md[20];
    unsigned int len = 0;
    HMAC_Init_ex(h, nullptr, 0, nullptr, nullptr);
    HMAC_Update(h, data, n);
    if (extra4) HMAC_Update(h, extra4, 4);
    HMAC_Final(h, md, &len);
    memcpy(out10, md, 10);
}

bool tag_ok(HMAC_CTX* h, const uint8_t* data, int n, const uint8_t* extra4, const uint8_t* want) {
    uint8_t t[10];
    tag(h, data, n, extra4, t);
    return CRYPTO_memcmp(t, want, 10) == 0;
}

int rtp_header_len(const uint8_t* p, int n) {
    if (n < 12 || (p[0] >> 6) != 2) return -1;
    int len = 12 + 4 * (p[0] & 15);
    if (p[0] & 0x10) {
        if (n < len + 4) return -1;
        len += 4 + 4 * ((p[len + 2] << 8) | p[len + 3]);
    }
    return len <= n ? len : -1;
}

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }
inline void put_be32(uint8_t* p, uint32_t v) {
    p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}

// Replay window check/update on a 48-bit (RTP) or 31-bit (RTCP) index.
bool replay_check(RecvState& r, uint64_t idx, bool commit) {
    if (r.max_index == 0 && r.window == 0) {
        if (commit) { r.max_index = idx; r.window = 1; }
        return true;
    }
    if (idx > r.max_index) {
        if (commit) {
            uint64_t d = idx - r.max_index;
            r.window = d >= 64 ? 1 : (r.window << d) | 1;
            r.max_index = idx;
        }
        return true;
    }
    uint64_t d = r.max_index - idx;
    if (d >= 64) return false;
    if (r.window & (1ull << d)) return false;
    if (commit) r.window |= 1ull << d;
    return true;
}

// ---------------------------------------------------------------------------
// H.264 RFC 6184 packetisation
struct Nal {
    const uint8_t* p;
    int n;
};

std::vector<Nal> split_annexb(const uint8_t* b, int n) {
    std::vector<Nal> v;
    int i = 0, start = -1;
    while (i + 2 < n) {
        if (b[i] == 0 && b[i + 1] == 0 && b[i + 2] == 1) {
            if (start >= 0) {
                int e = i;
                while (e > start && b[e - 1] == 0) e--;
                if (e > start) v.push_back({b + start, e - start});
            }
            i += 3;
            start = i;
        } else {
            i++;
        }
    }
    if (start >= 0 && start < n) {
        int e = n;
        while (e > start && b[e - 1] == 0) e--;
        if (e > start) v.push_back({b + start, e - start});
    } else if (start < 0 && n > 0) {
        v.push_back({b, n});  // a bare NAL without start code
    }
    return v;
}

struct PacketWriter {
    Srtp* srtp;
    rtc_rtp_params* p;
    uint8_t* out;
    int cap, used = 0, count = 0;
    int* lens;
    int max_pkts;
    bool failed = false;

    int hdr() const { return p->playout_ext_id > 0 && p->playout_ext_id < 15 ? 20 : 12; }
    uint8_t* begin(int payload_len) {
        const int need = hdr() + payload_len + (srtp ? 10 : 0);
        if (count >= max_pkts || used + need > cap) {
            failed = true;
            return nullptr;
        }
        uint8_t* h = out + used;
        h[0] = 0x80;
        h[1] = p->payload_type & 0x7f;
        h[2] = p->seq >> 8;
        h[3] = p->seq & 0xff;
        put_be32(h + 4, p->timestamp);
        put_be32(h + 8, p->ssrc);
        if (hdr() == 20) {   // X bit, 0xBEDE one-byte profile, 1 word: [id|len-1=2][min 12b][max 12b]
            h[0] |= 0x10;
            h[12] = 0xBE;
            h[13] = 0xDE;
            h[14] = 0;
            h[15] = 1;
            const int mn = p->playout_min & 0xfff, mx = p->playout_max & 0xfff;
            h[16] = (uint8_t)((p->playout_ext_id << 4) | 2);
            h[17] = (uint8_t)(mn >> 4);
            h[18] = (uint8_t)(((mn & 15) << 4) | (mx >> 8));
            h[19] = (uint8_t)(mx & 0xff);
        }
        return h + hdr();
    }
    void end(int payload_len, bool marker) {
        uint8_t* h = out + used;
        if (marker) h[1] |= 0x80;
        int len = hdr() + payload_len;
        if (srtp) len = rtc_srtp_protect_rtp(srtp, h, len);
        lens[count++] = len;
        used += len;
        p->seq = (uint16_t)(p->seq + 1);
    }
};

}  // namespace

extern "C" {

// ---- DTLS ------------------------------------------------------------------
void* rtc_dtls_create(int role) {
    auto* d = new Dtls();
    d->role = role;
    if (!make_identity(d)) {
        d->err = "certificate generation failed: " + ssl_errors();
        d->state = 3;
        return d;
    }
    d->ctx = SSL_CTX_new(DTLS_method());
    SSL_CTX_set_min_proto_version(d->ctx, DTLS1_2_VERSION);
    SSL_CTX_use_certificate(d->ctx, d->cert);
    SSL_CTX_use_PrivateKey(d->ctx, d->key);
    SSL_CTX_set_verify(d->ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, verify_any);
    SSL_CTX_set_tlsext_use_srtp(d->ctx, "SRTP_AES128_CM_SHA1_80");  // returns 0 on success
    SSL_CTX_set_read_ahead(d->ctx, 1);
    d->ssl = SSL_new(d->ctx);
    BIO* bio = BIO_new(bio_method());
    BIO_set_data(bio, d);
    SSL_set_bio(d->ssl, bio, bio);
    SSL_set_options(d->ssl, SSL_OP_NO_QUERY_MTU);
    SSL_set_mtu(d->ssl, 1200 - 28);
    if (role) SSL_set_accept_state(d->ssl);
    else SSL_set_connect_state(d->ssl);
    return d;
}

void rtc_dtls_destroy(void* p) {
    auto* d = static_cast<Dtls*>(p);
    if (!d) return;
    if (d->ssl) SSL_free(d->ssl);
    if (d->ctx) SSL_CTX_free(d->ctx);
    if (d->cert) X509_free(d->cert);
    if (d->key) EVP_PKEY_free(d->key);
    delete d;
}

void rtc_dtls_set_role(void* p, int role) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state != 0 || !d->ssl) return;
    d->role = role;
    if (role) SSL_set_accept_state(d->ssl);
    else SSL_set_connect_state(d->ssl);
}

int rtc_dtls_fingerprint(void* p, char* out, int cap) {
    auto* d = static_cast<Dtls*>(p);
    int n = (int)d->local_fp.size();
    if (cap <= n) return -1;
    memcpy(out, d->local_fp.c_str(), n + 1);
    return n;
}

void rtc_dtls_set_remote_fingerprint(void* p, const char* fp) { static_cast<Dtls*>(p)->remote_fp = fp ? fp : ""; }

int rtc_dtls_start(void* p) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state == 3) return -1;
    if (d->state == 0) d->state = 1;
    if (d->role == 0) return handshake_step(d) < 0 ? -1 : 0;
    return 0;
}

int rtc_dtls_feed(void* p, const uint8_t* dgram, int n) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state >= 3) return -1;
    d->in.emplace_back(dgram, dgram + n);
    if (d->state < 2) {
        d->state = 1;
        int r = handshake_step(d);
        if (r != 0) {
            if (r == 1) drain_app(d);  // records that arrived with the final flight
            return r;
        }
        return 0;
    }
    drain_app(d);
    return 0;
}

int rtc_dtls_pop(void* p, uint8_t* out, int cap) {
    auto* d = static_cast<Dtls*>(p);
    if (d->out.empty()) return 0;
    Bytes& b = d->out.front();
    int n = (int)b.size();
    if (n > cap) return -1;
    memcpy(out, b.data(), n);
    d->out.pop_front();
    return n;
}

int rtc_dtls_read(void* p, uint8_t* out, int cap) {
    auto* d = static_cast<Dtls*>(p);
    if (d->app.empty()) return 0;
    Bytes& b = d->app.front();
    int n = (int)b.size();
    if (n > cap) return -1;
    memcpy(out, b.data(), n);
    d->app.pop_front();
    return n;
}

int rtc_dtls_write(void* p, const uint8_t* data, int n) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state != 2) return -1;
    int r = SSL_write(d->ssl, data, n);
    return r > 0 ? r : -1;
}

int rtc_dtls_state(void* p) { return static_cast<Dtls*>(p)->state; }

int rtc_dtls_timeout_ms(void* p) {
    auto* d = static_cast<Dtls*>(p);
    struct timeval tv;
    if (d->state != 1 || !DTLSv1_get_timeout(d->ssl, &tv)) return -1;
    return (int)(tv.tv_sec * 1000 + tv.tv_usec / 1000);
}

int rtc_dtls_on_timeout(void* p) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state != 1) return 0;
    return DTLSv1_handle_timeout(d->ssl);
}

int rtc_dtls_srtp_keys(void* p, uint8_t* local30, uint8_t* remote30) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state != 2) return -1;
    uint8_t m[60];
    static const char label[] = "EXTRACTOR-dtls_srtp";
    if (SSL_export_keying_material(d->ssl, m, sizeof m, label, sizeof label - 1, nullptr, 0, 0) != 1) return -1;
    const uint8_t *ck = m, *sk = m + 16, *cs = m + 32, *ss = m + 46;
    const bool server = d->role == 1;
    memcpy(local30, server ? sk : ck, 16);
    memcpy(local30 + 16, server ? ss : cs, 14);
    memcpy(remote30, server ? ck : sk, 16);
    memcpy(remote30 + 16, server ? cs : ss, 14);
    return 0;
}

const char* rtc_dtls_error(void* p) { return static_cast<Dtls*>(p)->err.c_str(); }

void rtc_dtls_close(void* p) {
    auto* d = static_cast<Dtls*>(p);
    if (d->state == 2) SSL_shutdown(d->ssl);
    d->state = 4;
}

// ---- SRTP ------------------------------------------------------------------
void* rtc_srtp_create(const uint8_t* ks) {
    auto* s = new Srtp();
    s->aes = EVP_CIPHER_CTX_new();
    const uint8_t *mk = ks, *ms = ks + 16;
    derive(s->aes, mk, ms, 0, s->rtp.enc, 16);
    derive(s->aes, mk, ms, 1, s->rtp.auth, 20);
    derive(s->aes, mk, ms, 2, s->rtp.salt, 14);
    derive(s->aes, mk, ms, 3, s->rtcp.enc, 16);
    derive(s->aes, mk, ms, 4, s->rtcp.auth, 20);
    derive(s->aes, mk, ms, 5, s->rtcp.salt, 14);
    s->hm_rtp = HMAC_CTX_new();
    s->hm_rtcp = HMAC_CTX_new();
    HMAC_Init_ex(s->hm_rtp, s->rtp.auth, 20, EVP_sha1(), nullptr);
    HMAC_Init_ex(s->hm_rtcp, s->rtcp.auth, 20, EVP_sha1(), nullptr);
    return s;
}

void rtc_srtp_destroy(void* p) {
    auto* s = static_cast<Srtp*>(p);
    if (!s) return;
    EVP_CIPHER_CTX_free(s->aes);
    HMAC_CTX_free(s->hm_rtp);
    HMAC_CTX_free(s->hm_rtcp);
    delete s;
}

void rtc_srtp_session_keys(void* p, uint8_t* o) {
    auto* s = static_cast<Srtp*>(p);
    const Keys* k[2] = {&s->rtp, &s->rtcp};
    for (int i = 0; i < 2; i++, o += 50) {
        memcpy(o, k[i]->enc, 16);
        memcpy(o + 16, k[i]->auth, 20);
        memcpy(o + 36, k[i]->salt, 14);
    }
}

int rtc_srtp_protect_rtp(void* p, uint8_t* pkt, int n) {
    auto* s = static_cast<Srtp*>(p);
    int hl = rtp_header_len(pkt, n);
    if (hl < 0) return -3;
    const uint32_t ssrc = be32(pkt + 8);
    const uint16_t seq = (uint16_t)(pkt[2] << 8 | pkt[3]);
    auto it = s->send_roc.find(ssrc);
    if (it == s->send_roc.end()) it = s->send_roc.emplace(ssrc, std::make_pair(0u, -1)).first;
    auto& st = it->second;
    // sender ROC: bump when the sequence number wraps (retransmissions of older packets keep theirs)
    uint32_t roc = st.first;
    if (st.second >= 0) {
        int d = (int)seq - st.second;
        if (d < -32768) st.first = ++roc;
        else if (d > 32768 && roc > 0) roc -= 1;  // late retransmission from before the wrap
    }
    if (st.second < 0 || (int16_t)(seq - (uint16_t)st.second) > 0) st.second = seq;
    const uint64_t index = ((uint64_t)roc << 16) | seq;
    uint8_t iv[16];
    packet_iv(s->rtp.salt, ssrc, index, iv);
    aes_cm(s->aes, s->rtp.enc, iv, pkt + hl, n - hl);
    uint8_t r[4];
    put_be32(r, roc);
    tag(s->hm_rtp, pkt, n, r, pkt + n);
    return n + 10;
}

int rtc_srtp_unprotect_rtp(void* p, uint8_t* pkt, int n) {
    auto* s = static_cast<Srtp*>(p);
    if (n < 12 + 10) return -3;
    const int m = n - 10;
    int hl = rtp_header_len(pkt, m);
    if (hl < 0) return -3;
    const uint32_t ssrc = be32(pkt + 8);
    const uint16_t seq = (uint16_t)(pkt[2] << 8 | pkt[3]);
    RecvState& r = s->recv[ssrc];
    if (!r.init) {
        r.init = true;
        r.s_l = seq;
        r.roc = 0;
    }
    uint32_t v;
    if (r.s_l < 32768) v = (seq - r.s_l > 32768) ? r.roc - 1 : r.roc;
    else v = (r.s_l - 32768 > seq) ? r.roc + 1 : r.roc;
    const uint64_t index = ((uint64_t)v << 16) | seq;
    uint8_t rb[4];
    put_be32(rb, v);
    if (!tag_ok(s->hm_rtp, pkt, m, rb, pkt + m)) return -1;
    if (!replay_check(r, index + 1, false)) return -2;
    replay_check(r, index + 1, true);
    if (v == r.roc + 1) {
        r.roc = v;
        r.s_l = seq;
    } else if (v == r.roc && seq > r.s_l) {
        r.s_l = seq;
    }
    uint8_t iv[16];
    packet_iv(s->rtp.salt, ssrc, index, iv);
    aes_cm(s->aes, s->rtp.enc, iv, pkt + hl, m - hl);
    return m;
}

int rtc_srtp_protect_rtcp(void* p, uint8_t* pkt, int n) {
    auto* s = static_cast<Srtp*>(p);
    if (n < 8) return -3;
    const uint32_t ssrc = be32(pkt + 4);
    uint32_t& idx = s->send_rtcp_index[ssrc];
    const uint32_t i = idx;
    idx = (idx + 1) & 0x7fffffff;
    uint8_t iv[16];
    packet_iv(s->rtcp.salt, ssrc, i, iv);
    aes_cm(s->aes, s->rtcp.enc, iv, pkt + 8, n - 8);
    put_be32(pkt + n, 0x80000000u | i);
    tag(s->hm_rtcp, pkt, n + 4, nullptr, pkt + n + 4);
    return n + 14;
}

int rtc_srtp_unprotect_rtcp(void* p, uint8_t* pkt, int n) {
    auto* s = static_cast<Srtp*>(p);
    if (n < 8 + 14) return -3;
    const int m = n - 14;
    if (!tag_ok(s->hm_rtcp, pkt, m + 4, nullptr, pkt + m + 4)) return -1;
    const uint32_t e_idx = be32(pkt + m);
    const uint32_t i = e_idx & 0x7fffffff;
    const uint32_t ssrc = be32(pkt + 4);
    RecvState& r = s->recv_rtcp[ssrc];
    if (!replay_check(r, (uint64_t)i + 1, false)) return -2;
    replay_check(r, (uint64_t)i + 1, true);
    if (e_idx & 0x80000000u) {
        uint8_t iv[16];
        packet_iv(s->rtcp.salt, ssrc, i, iv);
        aes_cm(s->aes, s->rtcp.enc, iv, pkt + 8, m - 8);
    }
    return m;
}

// ---- RTP packetisation -------------------------------------------------------
int rtc_h264_packetize(void* srtp, const uint8_t* annexb, int n, rtc_rtp_params* p, uint8_t* out, int cap,
                       int* lens, int max_pkts) {
    PacketWriter w{static_cast<Srtp*>(srtp), p, out, cap, 0, 0, lens, max_pkts};
    const int maxp = p->mtu - ((p->playout_ext_id > 0 && p->playout_ext_id < 15) ? 20 : 12);
    if (maxp < 64) return -1;
    std::vector<Nal> nals = split_annexb(annexb, n);
    const size_t nn = nals.size();
    for (size_t i = 0; i < nn;) {
        // STAP-A: aggregate a run of NALs that fits in one packet
        size_t j = i;
        int agg = 1;
        while (j < nn && agg + 2 + nals[j].n <= maxp) agg += 2 + nals[j++].n;
        if (j - i >= 2) {
            uint8_t* pl = w.begin(agg);
            if (!pl) return -1;
            uint8_t f = 0, nri = 0;
            int o = 1;
            for (size_t k = i; k < j; k++) {
                f |= nals[k].p[0] & 0x80;
                nri = nri > (nals[k].p[0] & 0x60) ? nri : (nals[k].p[0] & 0x60);
                pl[o] = nals[k].n >> 8;
                pl[o + 1] = nals[k].n & 0xff;
                memcpy(pl + o + 2, nals[k].p, nals[k].n);
                o += 2 + nals[k].n;
            }
            pl[0] = f | nri | 24;
            w.end(agg, j == nn);
            i = j;
            continue;
        }
        const Nal& nal = nals[i];
        if (nal.n <= maxp) {  // single NAL unit packet
            uint8_t* pl = w.begin(nal.n);
            if (!pl) return -1;
            memcpy(pl, nal.p, nal.n);
            w.end(nal.n, i + 1 == nn);
        } else {  // FU-A
            const uint8_t hdr = nal.p[0];
            const int chunk = maxp - 2;
            for (int off = 1; off < nal.n; off += chunk) {
                const int len = nal.n - off < chunk ? nal.n - off : chunk;
                uint8_t* pl = w.begin(len + 2);
                if (!pl) return -1;
                const bool first = off == 1, last = off + len >= nal.n;
                pl[0] = (hdr & 0xe0) | 28;
                pl[1] = (first ? 0x80 : 0) | (last ? 0x40 : 0) | (hdr & 0x1f);
                memcpy(pl + 2, nal.p + off, len);
                w.end(len + 2, last && i + 1 == nn);
            }
        }
        i++;
    }
    return w.failed ? -1 : w.count;
}

// H.265 RFC 7798 packetisation: single NAL unit packets, aggregation packets (AP,
// type 48) for runs of small NAL units (parameter sets), fragmentation units (FU,
// type 49) for NAL units larger than the MTU. The 2-byte payload headers keep the
// NAL's F bit, layer id and temporal id (AP: F = OR, layer / TID = minimum).
int rtc_h265_packetize(void* srtp, const uint8_t* annexb, int n, rtc_rtp_params* p, uint8_t* out, int cap,
                       int* lens, int max_pkts) {
    PacketWriter w{static_cast<Srtp*>(srtp), p, out, cap, 0, 0, lens, max_pkts};
    const int maxp = p->mtu - ((p->playout_ext_id > 0 && p->playout_ext_id < 15) ? 20 : 12);
    if (maxp < 64) return -1;
    std::vector<Nal> nals = split_annexb(annexb, n);
    const size_t nn = nals.size();
    for (size_t i = 0; i < nn;) {
        if (nals[i].n < 3) { i++; continue; }
        size_t j = i;
        int agg = 2;
        while (j < nn && nals[j].n >= 3 && agg + 2 + nals[j].n <= maxp) agg += 2 + nals[j++].n;
        if (j - i >= 2) {
            uint8_t* pl = w.begin(agg);
            if (!pl) return -1;
            int f = 0, layer = 63, tid = 7;
            int o = 2;
            for (size_t k = i; k < j; k++) {
                const uint8_t* h = nals[k].p;
                f |= h[0] & 0x80;
                const int ly = ((h[0] & 1) << 5) | (h[1] >> 3), t = h[1] & 7;
                layer = ly < layer ? ly : layer;
                tid = t < tid ? t : tid;
                pl[o] = nals[k].n >> 8;
                pl[o + 1] = nals[k].n & 0xff;
                memcpy(pl + o + 2, nals[k].p, nals[k].n);
                o += 2 + nals[k].n;
            }
            pl[0] = (uint8_t)(f | (48 << 1) | (layer >> 5));
            pl[1] = (uint8_t)(((layer & 31) << 3) | tid);
            w.end(agg, j == nn);
            i = j;
            continue;
        }
        const Nal& nal = nals[i];
        if (nal.n <= maxp) {
            uint8_t* pl = w.begin(nal.n);
            if (!pl) return -1;
            memcpy(pl, nal.p, nal.n);
            w.end(nal.n, i + 1 == nn);
        } else {
            const uint8_t h0 = nal.p[0], h1 = nal.p[1];
            const int type = (h0 >> 1) & 63;
            const int chunk = maxp - 3;
            for (int off = 2; off < nal.n; off += chunk) {
                const int len = nal.n - off < chunk ? nal.n - off : chunk;
                uint8_t* pl = w.begin(len + 3);
                if (!pl) return -1;
                const bool first = off == 2, last = off + len >= nal.n;
                pl[0] = (uint8_t)((h0 & 0x81) | (49 << 1));
                pl[1] = h1;
                pl[2] = (uint8_t)((first ? 0x80 : 0) | (last ? 0x40 : 0) | type);
                memcpy(pl + 3, nal.p + off, len);
                w.end(len + 3, last && i + 1 == nn);
            }
        }
        i++;
    }
    return w.failed ? -1 : w.count;
}

// AV1 RTP payload (AOM "RTP Payload Format for AV1" v1.0): one temporal unit of
// low-overhead OBUs (obu_has_size_field = 1, as av1_cpu.cpp writes them) -> packets.
// Aggregation header |Z|Y|W=0|N|000|: every OBU element carries a LEB128 length;
// temporal delimiters, tile lists and padding are dropped, the OBU size field is
// removed (the element length replaces it); OBUs larger than a packet are split
// (Y on the packet holding the head, Z on the packets continuing it); N on the first
// packet of a temporal unit with a sequence header. Marker = last packet of the TU.
static int leb128_len(uint32_t v) {
    int n = 1;
    while (v >= 0x80) {
        v >>= 7;
        n++;
    }
    return n;
}
static int put_leb128(uint8_t* d, uint32_t v) {
    int n = 0;
    do {
        uint8_t b = v & 0x7f;
        v >>= 7;
        d[n++] = (uint8_t)(b | (v ? 0x80 : 0));
    } while (v);
    return n;
}

int rtc_av1_packetize(void* srtp, const uint8_t* tu, int n, rtc_rtp_params* p, uint8_t* out, int cap, int* lens,
                      int max_pkts) {
    PacketWriter w{static_cast<Srtp*>(srtp), p, out, cap, 0, 0, lens, max_pkts};
    const int maxp = p->mtu - ((p->playout_ext_id > 0 && p->playout_ext_id < 15) ? 20 : 12);
    if (maxp < 64) return -1;
    struct Elem { uint8_t hdr[2]; int hlen; const uint8_t* pl; int plen; };
    std::vector<Elem> el;
    bool seq = false;
    for (int pos = 0; pos < n;) {   // parse the OBUs
        const uint8_t h0 = tu[pos];
        const int type = (h0 >> 3) & 15, ext = (h0 >> 2) & 1, has_size = (h0 >> 1) & 1;
        int q = pos + 1 + ext;
        if (q > n) return -1;
        uint64_t sz = 0;
        if (has_size) {
            int sh = 0;
            for (;;) {
                if (q >= n || sh > 56) return -1;
                const uint8_t b = tu[q++];
                sz |= (uint64_t)(b & 0x7f) << sh;
                sh += 7;
                if (!(b & 0x80)) break;
            }
        } else {
            sz = (uint64_t)(n - q);
        }
        if (q + (int64_t)sz > n) return -1;
        if (type == 1) seq = true;
        if (type != 2 && type != 8 && type != 15) {
            Elem e;
            e.hdr[0] = (uint8_t)(h0 & ~2);
            e.hdr[1] = ext ? tu[pos + 1] : 0;
            e.hlen = 1 + ext;
            e.pl = tu + q;
            e.plen = (int)sz;
            el.push_back(e);
        }
        pos = q + (int)sz;
    }
    if (el.empty()) return 0;
    // packetise: elements in order, split where a packet fills up
    std::vector<uint8_t> pk((size_t)maxp);
    int used = 1;          // aggregation header first
    bool z = false;        // this packet starts with a continuation
    bool first = true;
    auto flush = [&](bool y, bool last) -> bool {
        pk[0] = (uint8_t)((z ? 0x80 : 0) | (y ? 0x40 : 0) | ((first && seq) ? 0x08 : 0));
        uint8_t* d = w.begin(used);
        if (!d) return false;
        memcpy(d, pk.data(), (size_t)used);
        w.end(used, last);
        first = false;
        used = 1;
        return true;
    };
    for (size_t k = 0; k < el.size(); k++) {
        const Elem& e = el[k];
        const int total = e.hlen + e.plen;   // element bytes (header + payload)
        int off = 0;                         // bytes of this element already sent
        while (off < total) {
            const int rem = total - off;
            const int room = maxp - used;
            if (leb128_len((uint32_t)rem) + rem <= room) {   // the rest fits
                used += put_leb128(pk.data() + used, (uint32_t)rem);
                for (int i = 0; i < rem; i++) {
                    const int b = off + i;
                    pk[(size_t)used + i] = b < e.hlen ? e.hdr[b] : e.pl[b - e.hlen];
                }
                used += rem;
                off = total;
                if (k + 1 == el.size()) {
                    if (!flush(false, true)) return -1;
                    z = false;
                }
            } else if (room >= 8) {   // a fragment fills the packet
                const int frag = room - leb128_len((uint32_t)room);
                used += put_leb128(pk.data() + used, (uint32_t)frag);
                for (int i = 0; i < frag; i++) {
                    const int b = off + i;
                    pk[(size_t)used + i] = b < e.hlen ? e.hdr[b] : e.pl[b - e.hlen];
                }
                used += frag;
                off += frag;
                if (!flush(true, false)) return -1;
                z = true;
            } else {   // no useful room left: close this packet before the element
                if (!flush(false, false)) return -1;
                z = false;
            }
        }
    }
    return w.failed ? -1 : w.count;
}

int rtc_rtp_packet(void* srtp, const uint8_t* payload, int n, rtc_rtp_params* p, uint8_t* out, int cap) {
    int len = 0;
    PacketWriter w{static_cast<Srtp*>(srtp), p, out, cap, 0, 0, &len, 1};
    uint8_t* pl = w.begin(n);
    if (!pl) return -1;
    memcpy(pl, payload, n);
    w.end(n, p->marker != 0);
    return len;
}

// ---- CRC32c (SCTP, RFC 4960 appendix B) --------------------------------------
uint32_t rtc_crc32c(const uint8_t* data, int n) {
    struct Tables {
        uint32_t t[8][256];
        Tables() {
            for (uint32_t i = 0; i < 256; i++) {
                uint32_t c = i;
                for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1)));
                t[0][i] = c;
            }
            for (int k = 1; k < 8; k++)
                for (uint32_t i = 0; i < 256; i++) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xff];
        }
    };
    static const Tables tabs;  // thread-safe one-time init
    const auto& table = tabs.t;
    uint32_t c = 0xffffffffu;
    int i = 0;
    for (; i + 8 <= n; i += 8) {  // slicing-by-8
        uint32_t lo, hi;
        memcpy(&lo, data + i, 4);
        memcpy(&hi, data + i + 4, 4);
        lo ^= c;
        c = table[7][lo & 0xff] ^ table[6][(lo >> 8) & 0xff] ^ table[5][(lo >> 16) & 0xff] ^ table[4][lo >> 24] ^
            table[3][hi & 0xff] ^ table[2][(hi >> 8) & 0xff] ^ table[1][(hi >> 16) & 0xff] ^ table[0][hi >> 24];
    }
    for (; i < n; i++) c = (c >> 8) ^ table[0][(c ^ data[i]) & 0xff];
    return ~c;
}

}  // extern "C"
