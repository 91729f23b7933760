// WebRTC-mode client core (reference addons/gst-web/src/{signaling.js,
// webrtc.js,app.js}, SURVEY C38): GStreamer-demo signalling over a websocket,
// two RTCPeerConnections answering the server's offers (video + "input" data
// channel as peer 1, audio alone as peer 3: app.js:375-378), answer-SDP munging
// (webrtc.js:271-320), the "input" data channel carrying the same input
// vocabulary as the websocket mode, the server's {"type":..., "data":...}
// telemetry/control messages and getStats reports (webrtc.js:494).

export class Signalling {
  // peerId 1 is the browser; the streaming server registers as 0 and calls us.
  constructor(url, peerId = 1, WebSocketImpl = globalThis.WebSocket) {
    this.url = url;
    this.peerId = peerId;
    this.WS = WebSocketImpl;
    this.ws = null;
    this.onsdp = () => {};
    this.onice = () => {};
    this.onstatus = () => {};
    this.onerror = () => {};
    this.ondisconnect = () => {};
    this.retryMs = 3000;
  }

  connect(meta) {
    this.ws = new this.WS(this.url);
    this.ws.onopen = () => {
      const m = meta ? ' ' + btoa(JSON.stringify(meta)) : '';
      this.ws.send(`HELLO ${this.peerId}${m}`);
      this.onstatus('registering');
    };
    this.ws.onmessage = (ev) => this.handle(ev.data);
    this.ws.onclose = () => {
      this.ondisconnect();
      setTimeout(() => this.connect(meta), this.retryMs);
    };
    this.ws.onerror = (e) => this.onerror(e);
  }

  handle(data) {
    if (data === 'HELLO') { this.onstatus('registered, waiting for the stream'); return; }
    if (data.startsWith('SESSION_OK')) { this.onstatus('session started'); return; }
    if (data.startsWith('ERROR')) { this.onerror(new Error(data)); return; }
    let msg;
    try { msg = JSON.parse(data); } catch (e) { this.onerror(new Error('bad message: ' + data)); return; }
    if (msg.sdp) this.onsdp(msg.sdp);
    else if (msg.ice) this.onice(msg.ice);
  }

  sendSdp(desc) { this.ws.send(JSON.stringify({ sdp: { type: desc.type, sdp: desc.sdp } })); }

  sendIce(c) { this.ws.send(JSON.stringify({ ice: { candidate: c.candidate, sdpMLineIndex: c.sdpMLineIndex } })); }
}

// Parses a server data-channel message into {type, data}; "system" actions are
// split into [name, value] (gstwebrtc_app.py send_framerate / send_encoder / ...).
export function parseServerMessage(text) {
  let msg;
  try { msg = JSON.parse(text); } catch (e) { return null; }
  if (!msg || typeof msg.type !== 'string') return null;
  if (msg.type === 'system' && msg.data && typeof msg.data.action === 'string') {
    const i = msg.data.action.indexOf(',');
    msg.action = i < 0 ? [msg.data.action, ''] : [msg.data.action.slice(0, i), msg.data.action.slice(i + 1)];
  }
  return msg;
}

// Answer-SDP munging before setLocalDescription (the browser's defaults are not what a
// desktop stream wants): H.264 parameter sets travel with every IDR
// (sps-pps-idr-in-keyframe=1), and unless the session uses multiopus, Opus is stereo
// with 10 ms packets (stereo=1, minptime=10). Existing values are overridden, missing
// ones are inserted before the fmtp parameter they belong with.
export function mungeAnswerSdp(sdp) {
  const set = (text, key, value, anchor, present) => {
    if (new RegExp(`[^-]${key}=${value}[^\\d]`).test(text) || !new RegExp(`[^-]${anchor}=`).test(text)) return text;
    if (present.test(text)) return text.replace(new RegExp(`${key}=\\d+`, 'g'), `${key}=${value}`);
    return text.split(`${anchor}=`).join(`${key}=${value};${anchor}=`);
  };
  let out = set(sdp, 'sps-pps-idr-in-keyframe', '1', 'packetization-mode', /[^-]sps-pps-idr-in-keyframe=\d+/);
  if (out.indexOf('multiopus') === -1) {
    out = set(out, 'stereo', '1', 'useinbandfec', /[^-]stereo=\d+/);
    out = set(out, 'minptime', '10', 'useinbandfec', /[^-]minptime=\d+/);
  }
  return out;
}

// Flattens an RTCStatsReport into the server's _stats_video / _stats_audio payloads:
// the inbound-rtp entry of the kind, its codec, and the selected candidate pair.
export function summariseStats(report, kind) {
  const byId = new Map();
  report.forEach((s) => byId.set(s.id, s));
  const out = {};
  report.forEach((s) => {
    if (s.type === 'inbound-rtp' && s.kind === kind) {
      Object.assign(out, s);
      const codec = s.codecId && byId.get(s.codecId);
      if (codec) out.codec = { mimeType: codec.mimeType, clockRate: codec.clockRate, sdpFmtpLine: codec.sdpFmtpLine };
    }
    if (s.type === 'candidate-pair' && (s.selected || s.nominated) && s.state === 'succeeded') {
      out.transport = { currentRoundTripTime: s.currentRoundTripTime, availableIncomingBitrate: s.availableIncomingBitrate,
        bytesReceived: s.bytesReceived };
    }
  });
  return out;
}

export class WebRTCClient {
  // media: 'video' (peer 1: video + input channel) or 'audio' (peer 3: audio only); the
  // element is the <video> or <audio> the remote track plays in.
  constructor(video, signalling, rtcConfig = {}, RTCPeerConnectionImpl = globalThis.RTCPeerConnection, media = 'video') {
    this.video = video;
    this.media = media;
    this.sig = signalling;
    this.rtcConfig = rtcConfig;
    this.PC = RTCPeerConnectionImpl;
    this.pc = null;
    this.channel = null;
    this.onmessage = () => {};
    this.onstate = () => {};
    this.onchannelopen = () => {};
    this.state = { framerate: 0, videoBitrate: 0, audioBitrate: 0, encoder: '', resolution: '', latencyMs: 0 };
    this.sig.onsdp = (sdp) => this.onSdp(sdp);
    this.sig.onice = (ice) => this.onIce(ice);
  }

  async onSdp(sdp) {
    if (sdp.type !== 'offer') return;
    this.reset();
    this.pc = new this.PC(this.rtcConfig);
    this.pc.ontrack = (ev) => {
      if (ev.track.kind === this.media && this.video) {
        this.video.srcObject = ev.streams[0] || new MediaStream([ev.track]);
        this.video.play && this.video.play().catch(() => {});
      }
    };
    this.pc.onicecandidate = (ev) => { if (ev.candidate) this.sig.sendIce(ev.candidate); };
    this.pc.onconnectionstatechange = () => this.onstate(this.pc.connectionState);
    this.pc.ondatachannel = (ev) => this.bindChannel(ev.channel);
    await this.pc.setRemoteDescription(sdp);
    const answer = await this.pc.createAnswer();
    await this.pc.setLocalDescription({ type: answer.type, sdp: mungeAnswerSdp(answer.sdp) });
    this.sig.sendSdp(this.pc.localDescription);
  }

  async onIce(ice) {
    if (this.pc && ice && ice.candidate) {
      try { await this.pc.addIceCandidate(ice); } catch (e) { /* late candidate after close */ }
    }
  }

  bindChannel(ch) {
    this.channel = ch;
    ch.onopen = () => this.onchannelopen();
    ch.onmessage = (ev) => {
      const msg = parseServerMessage(ev.data);
      if (!msg) return;
      if (msg.action) {
        const [name, value] = msg.action;
        if (name === 'framerate') this.state.framerate = parseInt(value, 10);
        else if (name === 'video_bitrate') this.state.videoBitrate = parseInt(value, 10);
        else if (name === 'audio_bitrate') this.state.audioBitrate = parseInt(value, 10);
        else if (name === 'encoder') this.state.encoder = value;
        else if (name === 'resolution') this.state.resolution = value;
      } else if (msg.type === 'ping') {
        this.send('pong,' + msg.data.start_time);
      } else if (msg.type === 'latency_measurement') {
        this.state.latencyMs = msg.data.latency_ms;
      }
      this.onmessage(msg);
    };
  }

  send(text) {
    if (this.channel && this.channel.readyState === 'open') this.channel.send(text);
  }

  setVideoBitrate(kbps) { this.send(`vb,${kbps | 0}`); }
  setAudioBitrate(bps) { this.send(`ab,${bps | 0}`); }
  setFramerate(fps) { this.send(`_arg_fps,${fps | 0}`); }
  requestResolution(w, h) { this.send(`r,${w & ~1}x${h & ~1}`); }
  setScaling(ratio) { this.send(`s,${ratio}`); }

  // Reports client-side stats (getStats) as _stats_video / _stats_audio JSON over this
  // peer's input channel; `audioPeer` (the separate audio connection) supplies the audio
  // half, as in the reference's two-peer client.
  async reportStats(audioPeer = null) {
    if (!this.pc || !this.pc.getStats) return;
    const video = summariseStats(await this.pc.getStats(), 'video');
    let audio = summariseStats(await this.pc.getStats(), 'audio');
    if (audioPeer && audioPeer.pc && audioPeer.pc.getStats) audio = summariseStats(await audioPeer.pc.getStats(), 'audio');
    if (video.framesPerSecond !== undefined) this.send(`_f,${Math.round(video.framesPerSecond)}`);
    this.send('_stats_video,' + JSON.stringify(video));
    this.send('_stats_audio,' + JSON.stringify(audio));
    return { video, audio };
  }

  reset() {
    if (this.channel) { try { this.channel.close(); } catch (e) { /* closed */ } }
    if (this.pc) { try { this.pc.close(); } catch (e) { /* closed */ } }
    this.channel = null;
    this.pc = null;
  }
}
