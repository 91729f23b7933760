// C ABI of the native WebRTC transport core (libselkies_rtc.so).
//
// The reference's WebRTC mode runs media through GStreamer webrtcbin
// (legacy/gstwebrtc_app.py:808-1000) or the vendored aiortc stack
// (webrtc/rtcdtlstransport.py, webrtc/rtcrtpsender.py, webrtc/codecs/h264.py).
// Here the per-packet work — DTLS records, SRTP/SRTCP protection, RFC 6184
// H.264 packetisation and the SCTP CRC32c — is C++ on OpenSSL, called once per
// access unit; signalling, ICE, SCTP and RTCP control stay in Python
// (selkies_gstreamer_amd/webrtc/).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- DTLS (RFC 6347 + RFC 5764 use_srtp) ---------------------------------
// role: 1 = DTLS server (setup:passive), 0 = client (setup:active).
void* rtc_dtls_create(int role);
void rtc_dtls_destroy(void* d);
// Changes the role before the handshake starts (the certificate is kept, so the
// fingerprint already offered stays valid when the answer picks setup:passive).
void rtc_dtls_set_role(void* d, int role);
// "AB:CD:..." SHA-256 fingerprint of the local (self-signed ECDSA P-256) certificate.
int rtc_dtls_fingerprint(void* d, char* out, int cap);
// Expected remote fingerprint from the SDP (checked when the handshake completes).
void rtc_dtls_set_remote_fingerprint(void* d, const char* fp);
// Client: produce the first flight. Server: no-op.
int rtc_dtls_start(void* d);
// Feed one received datagram. Returns 1 when the handshake completed on this
// call, 0 otherwise, <0 on fatal error (see rtc_dtls_error).
int rtc_dtls_feed(void* d, const uint8_t* dgram, int n);
// Pops the next datagram to send into out; returns its length, 0 if none.
int rtc_dtls_pop(void* d, uint8_t* out, int cap);
// Application data (SCTP packets): read one received record / write one.
int rtc_dtls_read(void* d, uint8_t* out, int cap);
int rtc_dtls_write(void* d, const uint8_t* data, int n);
// 0 new, 1 handshaking, 2 connected, 3 failed, 4 closed
int rtc_dtls_state(void* d);
// Milliseconds until the retransmission timer fires (-1: none); on expiry call
// rtc_dtls_on_timeout and send what rtc_dtls_pop returns.
int rtc_dtls_timeout_ms(void* d);
int rtc_dtls_on_timeout(void* d);
// 30 bytes each: 16-byte master key + 14-byte master salt, for the local
// (sending) and remote (receiving) direction. Returns 0 on success.
int rtc_dtls_srtp_keys(void* d, uint8_t* local30, uint8_t* remote30);
const char* rtc_dtls_error(void* d);
void rtc_dtls_close(void* d);

// ---- SRTP / SRTCP, AES_CM_128_HMAC_SHA1_80 (RFC 3711) --------------------
void* rtc_srtp_create(const uint8_t* key_salt30);
void rtc_srtp_destroy(void* s);
// In place: pkt has room for n + 10 (RTP) / n + 14 (RTCP) bytes. Returns the new length, <0 on error.
int rtc_srtp_protect_rtp(void* s, uint8_t* pkt, int n);
int rtc_srtp_protect_rtcp(void* s, uint8_t* pkt, int n);
// In place; returns the plaintext length or <0 (-1 auth failure, -2 replay, -3 malformed).
int rtc_srtp_unprotect_rtp(void* s, uint8_t* pkt, int n);
int rtc_srtp_unprotect_rtcp(void* s, uint8_t* pkt, int n);
// Derived session keys (RFC 3711 §4.3, test hook): rtp enc16|auth20|salt14, rtcp enc16|auth20|salt14.
void rtc_srtp_session_keys(void* s, uint8_t* out100);

// ---- RTP packetisation ---------------------------------------------------
struct rtc_rtp_params {
    uint32_t ssrc;
    uint32_t timestamp;
    uint16_t seq;        // in: first sequence number; out: next one
    uint8_t payload_type;
    uint8_t marker;      // raw payloads only (H.264 sets it on the last packet)
    int mtu;             // max RTP packet size before SRTP (e.g. 1200)
    // playout-delay header extension (http://www.webrtc.org/experiments/rtp-hdrext/playout-delay,
    // one-byte form, RFC 8285) on every packet when ext id 1..14; delays in 10 ms units
    // (0/0 = render as soon as decoded). 0 = no extension.
    int playout_ext_id, playout_min, playout_max;
};
// Splits an Annex-B access unit into RFC 6184 packets (single NAL, STAP-A for
// runs of small NALs such as SPS+PPS, FU-A for large ones), optionally SRTP
// protects them (srtp may be NULL) and writes them back to back into out;
// lens[i] = length of packet i. Returns the packet count, <0 if out/lens are
// too small.
int rtc_h264_packetize(void* srtp, const uint8_t* annexb, int n, struct rtc_rtp_params* p, uint8_t* out,
                       int cap, int* lens, int max_pkts);
// RFC 7798 (H.265) packetisation: single NAL / AP / FU payloads, same contract.
int rtc_h265_packetize(void* srtp, const uint8_t* annexb, int n, struct rtc_rtp_params* p, uint8_t* out,
                       int cap, int* lens, int max_pkts);
// AV1 (AOM RTP payload format): one temporal unit of size-delimited OBUs.
int rtc_av1_packetize(void* srtp, const uint8_t* tu, int n, rtc_rtp_params* p, uint8_t* out, int cap, int* lens,
                      int max_pkts);
// One packet around an arbitrary payload (Opus, ...). Returns its length.
int rtc_rtp_packet(void* srtp, const uint8_t* payload, int n, struct rtc_rtp_params* p, uint8_t* out, int cap);

// ---- SCTP ---------------------------------------------------------------
uint32_t rtc_crc32c(const uint8_t* data, int n);

#ifdef __cplusplus
}
#endif
