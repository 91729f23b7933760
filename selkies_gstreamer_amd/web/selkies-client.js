// Browser client for the MI355X streaming server (data websocket protocol of
// server/protocol.py). Connects, sends SETTINGS, decodes H.264 / JPEG stripes
// with WebCodecs, plays Opus audio, forwards input, ACKs frames every 50 ms,
// reports client fps, handles clipboard, uploads, cursor, multi-display hashes.
import { AudioPipeline } from './lib/audio.js';
import {
  ControlApi, FallbackPolicy, ImeComposer, SAFE_DEFAULTS, SharedProbe,
} from './lib/control.js';
import { Dashboard, parseRole } from './lib/dashboard.js';
import { Input } from './lib/input.js';
import {
  b64decode, b64ToUtf8, evenDown, parseFrame, parseText, utf8ToB64,
} from './lib/protocol.js';
import { VideoRenderer } from './lib/video.js';

const ACK_INTERVAL_MS = 50;
const METRICS_INTERVAL_MS = 1000;
const UPLOAD_CHUNK = 64 * 1024;
const STORAGE_KEY = 'selkies-mi355x-settings';

const $ = (id) => document.getElementById(id);

class Client {
  constructor() {
    this.canvas = $('stream');
    this.video = new VideoRenderer(this.canvas, (e) => this.onDecoderError(e), () => this.sendText('REQUEST_KEYFRAME'));
    this.audio = new AudioPipeline();
    this.input = new Input(this.canvas, (m) => this.sendText(m), () => [this.canvas.width, this.canvas.height]);
    this.input.onMenuHotkey = () => $('sidebar').classList.toggle('open');          // Ctrl+Shift+M
    this.input.onFullscreenHotkey = () => document.documentElement.requestFullscreen();   // Ctrl+Shift+F
    this.ws = null;
    this.killed = false;
    this.serverSettings = {};
    this.settings = this.loadSettings();
    this.display = this.parseHash();
    this.clipParts = null;
    this.timers = [];
    this.lastMetrics = performance.now();
    this.stats = {};
    this.control = new ControlApi(this);
    this.fallback = new FallbackPolicy();
    this.probe = this.display.shared ? new SharedProbe() : null;
    this.ime = new ImeComposer((m) => this.sendText(m));
  }

  // ---------------------------------------------------------------- control API host
  get shared() { return !!this.display.shared; }
  get displayId() { return this.display.id; }
  post(obj) { window.postMessage(obj, window.location.origin); }
  saveSetting(name, value) { this.settings[name] = value; this.saveSettings(); }
  applySettings(obj) {
    Object.assign(this.settings, obj);
    this.saveSettings();
    this.syncUi();
    this.sendText(this.settingsMessage());
  }
  setManualResolution(w, h) {
    Object.assign(this.settings, { is_manual_resolution_mode: true, manual_width: w, manual_height: h });
    this.saveSettings();
    this.video.reset();
    this.sendText(`r,${w}x${h},${this.display.id}`);
  }
  resetResolution() {
    Object.assign(this.settings, { is_manual_resolution_mode: false, manual_width: 0, manual_height: 0 });
    this.saveSettings();
    this.video.reset();
    const dpr = this.settings.use_css_scaling ? 1 : (window.devicePixelRatio || 1);
    this.sendText(`r,${evenDown(window.innerWidth * dpr)}x${evenDown(window.innerHeight * dpr)},${this.display.id}`);
  }
  clearVideo() { this.video.reset(); this.video.resize(this.canvas.width, this.canvas.height); }
  startMic() { this.audio.startMic((b) => this.sendBinary(b)); }
  stopMic() { this.audio.stopMic(); }
  audioOn(on) { if (on) this.audio.start(); else this.audio.stop(); }
  selectAudioDevice(context, deviceId) {
    if (context === 'output') this.audio.setOutputDevice && this.audio.setOutputDevice(deviceId);
    else { this.settings.mic_device = deviceId; this.saveSettings(); }
  }
  setGamepads(on) { this.input.gamepadsEnabled = on; }
  setTrackpad(on) { this.input.trackpad = on; }
  setSynth(v) { this.input.synth = v; }
  showKeyboard() { const k = $('keyboard-input-assist'); if (k) { k.value = ''; k.focus(); } }
  fullscreen() { document.documentElement.requestFullscreen(); }
  setClipboard(text) { this.clipboardOut(text); }
  updateRendering() {
    this.canvas.style.imageRendering = this.settings.anti_aliasing === false ? 'pixelated' : 'auto';
  }

  // Decoder errors: transient ones are survived (the stripe decoder is recreated at the
  // next keyframe); repeated ones reset to SAFE_DEFAULTS and reload (FallbackPolicy).
  onDecoderError(e) {
    this.status(`decoder error: ${e.message || e}`);
    const act = this.fallback.onError(performance.now(), this.shared);
    if (!act) return;
    if (act.resetSettings) { Object.assign(this.settings, SAFE_DEFAULTS); this.saveSettings(); }
    this.status('video decoding keeps failing: resetting to default settings and reloading');
    this.killed = true;
    if (this.ws) this.ws.close();
    setTimeout(() => window.location.reload(), act.reloadAfterMs);
  }

  // ---------------------------------------------------------------- settings
  loadSettings() {
    const defaults = { encoder: 'x264enc-striped', framerate: 60, h264_crf: 25, jpeg_quality: 40,
      paint_over_jpeg_quality: 90, h264_fullcolor: false, h264_streaming_mode: false, use_cpu: false,
      use_paint_over_quality: true, h264_paintover_crf: 18, h264_paintover_burst_frames: 5, audio_bitrate: 320000,
      is_manual_resolution_mode: false, manual_width: 0, manual_height: 0, scaling_dpi: 96,
      enable_binary_clipboard: false, use_css_scaling: false };
    try {
      return Object.assign(defaults, JSON.parse(localStorage.getItem(STORAGE_KEY) || '{}'));
    } catch (e) {
      return defaults;
    }
  }

  saveSettings() { localStorage.setItem(STORAGE_KEY, JSON.stringify(this.settings)); }

  parseHash() {
    // #display2[-left|-right|-up|-down], #shared (view only), #player2..4 (gamepads only)
    const role = parseRole(location.hash);
    if (role.player > 1) {
      this.input.padOffset = role.player - 1;
      this.input.gamepadOnly = true;
    }
    return role;
  }

  settingsMessage() {
    const dpr = this.settings.use_css_scaling ? 1 : (window.devicePixelRatio || 1);
    const s = Object.assign({}, this.settings, {
      initialClientWidth: evenDown(window.innerWidth * dpr),
      initialClientHeight: evenDown(window.innerHeight * dpr),
      displayId: this.display.id, displayPosition: this.display.position,
    });
    return `SETTINGS,${JSON.stringify(s)}`;
  }

  applyServerSettings(st) {
    this.serverSettings = st;
    const pick = (name, el) => {
      const def = st[name];
      const node = $(el);
      if (!def || !node) return;
      if ('min' in def) { node.min = def.min; node.max = def.max; if (def.min === def.max) node.disabled = true; }
      if (def.allowed && node.tagName === 'SELECT') {
        node.innerHTML = def.allowed.map((v) => `<option value="${v}">${v}</option>`).join('');
      }
      if ('locked' in def && def.locked) node.disabled = true;
    };
    pick('encoder', 'encoder');
    pick('framerate', 'framerate');
    pick('h264_crf', 'crf');
    pick('jpeg_quality', 'jpegq');
    if (st.encoder && st.encoder.allowed && !st.encoder.allowed.includes(this.settings.encoder)) {
      this.settings.encoder = st.encoder.value;
    }
    if (st.ui_title) document.title = st.ui_title.value;
    if (this.dashboard) this.dashboard.apply(st);
    this.syncUi();
  }

  syncUi() {
    if (this.video) {   // the stream's codec follows the negotiated encoder (lib/video.js codecString)
      this.video.encoder = this.settings.encoder;
      this.video.fps = Number(this.settings.framerate) || 60;
    }
    $('encoder').value = this.settings.encoder;
    $('framerate').value = this.settings.framerate;
    $('crf').value = this.settings.h264_crf;
    $('jpegq').value = this.settings.jpeg_quality;
    $('fullcolor').checked = !!this.settings.h264_fullcolor;
    $('framerate-v').textContent = this.settings.framerate;
    $('crf-v').textContent = this.settings.h264_crf;
    $('jpegq-v').textContent = this.settings.jpeg_quality;
  }

  updateSetting(name, value) {
    this.settings[name] = value;
    this.saveSettings();
    this.syncUi();
    if (this.ws && this.ws.readyState === 1) this.ws.send(this.settingsMessage());
  }

  // ---------------------------------------------------------------- connection
  connect() {
    const proto = location.protocol === 'https:' ? 'wss:' : 'ws:';
    const path = location.pathname.replace(/[^/]*$/, '') + 'websocket';
    this.ws = new WebSocket(`${proto}//${location.host}${path}`);
    this.ws.binaryType = 'arraybuffer';
    this.status('connecting');
    this.ws.onopen = () => this.status('connected');
    this.ws.onmessage = (ev) => (typeof ev.data === 'string' ? this.onText(ev.data) : this.onBinary(ev.data));
    this.ws.onclose = () => {
      this.stopTimers();
      this.input.detach();
      this.video.reset();
      if (this.killed) return;
      this.status('disconnected - reconnecting');
      setTimeout(() => this.connect(), 2000);
    };
  }

  sendText(m) { if (this.ws && this.ws.readyState === 1) this.ws.send(m); }
  sendBinary(b) { if (this.ws && this.ws.readyState === 1) this.ws.send(b); }

  startTimers() {
    this.stopTimers();
    this.timers.push(setInterval(() => {
      if (this.video.lastFrameId >= 0 && !this.display.shared) this.sendText(`CLIENT_FRAME_ACK ${this.video.lastFrameId}`);
    }, ACK_INTERVAL_MS));
    this.timers.push(setInterval(() => {
      const now = performance.now();
      const fps = this.video.takeFps(now - this.lastMetrics);
      this.lastMetrics = now;
      this.stats.fps = Math.round(fps);
      if (!this.display.shared) this.sendText(`_f,${Math.round(fps)}`);
      this.renderStats();
    }, METRICS_INTERVAL_MS));
    if (this.probe) {
      this.timers.push(setInterval(() => {
        for (const m of this.probe.tick(performance.now())) this.sendText(m);
        if (this.probe.state === 'error') this.status('no video from the shared session');
      }, 500));
    }
  }

  statsSnapshot() { return Object.assign({}, this.stats, { state: this.control.state }); }

  stopTimers() {
    for (const t of this.timers) clearInterval(t);
    this.timers = [];
  }

  onText(msg) {
    const m = parseText(msg);
    switch (m.kind) {
      case 'mode':
        if (!this.display.shared) this.sendText(this.settingsMessage());
        else { this.sendText('STOP_VIDEO'); this.sendText('START_VIDEO'); this.probe.reset(performance.now()); }
        if (this.display.player > 0) this.input.attach();   // view-only links send no input
        this.startTimers();
        break;
      case 'json': this.onJson(m.data); break;
      case 'kill':
        this.killed = true;
        this.status(`disconnected by server: ${m.reason}`);
        break;
      case 'reset': this.video.reset(); break;
      case 'cursor': this.setCursor(m.data); break;
      case 'clipboard': this.clipboardIn(m.mime, b64decode(m.b64)); break;
      case 'clipboard_start': this.clipParts = { mime: m.mime, size: m.size, chunks: [] }; break;
      case 'clipboard_data': if (this.clipParts) this.clipParts.chunks.push(b64decode(m.b64)); break;
      case 'clipboard_finish':
        if (this.clipParts) {
          const total = this.clipParts.chunks.reduce((a, c) => a + c.length, 0);
          const buf = new Uint8Array(total);
          let o = 0;
          for (const c of this.clipParts.chunks) { buf.set(c, o); o += c.length; }
          this.clipboardIn(this.clipParts.mime, buf);
          this.clipParts = null;
        }
        break;
      case 'displays': this.stats.displays = m.data.displays.join(', '); this.renderStats(); break;
      case 'state': this.status(m.msg.toLowerCase().replace('_', ' ')); break;
      default: break;
    }
  }

  onJson(d) {
    switch (d.type) {
      case 'server_settings': this.applyServerSettings(d.settings); break;
      case 'stream_resolution': this.video.resize(d.width, d.height); this.video.reset(); break;
      case 'system_stats': this.stats.cpu = d.cpu_percent; this.stats.mem = d.mem_used / d.mem_total; break;
      case 'gpu_stats': this.stats.gpu = d.load; this.stats.vram = d.memory_used / d.memory_total; break;
      case 'network_stats': this.stats.mbps = d.bandwidth_mbps; this.stats.rtt = d.latency_ms; break;
      default: break;
    }
    this.renderStats();
  }

  onBinary(buf) {
    const pkt = parseFrame(buf);
    if (!pkt) return;
    if (this.probe && (pkt.type === 'h264' || pkt.type === 'jpeg')) this.probe.onVideo();
    if (pkt.type === 'audio') this.audio.opus(pkt.payload);
    else if (pkt.type === 'h264') {
      if (this.canvas.width < pkt.width || this.canvas.height < pkt.y + pkt.height) {
        this.video.resize(Math.max(this.canvas.width, pkt.width), Math.max(this.canvas.height, pkt.y + pkt.height));
      }
      this.video.h264(pkt);
    } else if (pkt.type === 'jpeg') this.video.jpeg(pkt);
  }

  setCursor(c) {
    if (!c.curdata) { this.canvas.style.cursor = 'none'; return; }
    this.canvas.style.cursor = `url(data:image/png;base64,${c.curdata}) ${c.hotx} ${c.hoty}, auto`;
  }

  // ---------------------------------------------------------------- clipboard / uploads
  async clipboardIn(mime, bytes) {
    try {
      if (mime === 'text/plain') {
        const text = new TextDecoder().decode(bytes);
        $('clip').value = text;
        if (navigator.clipboard && document.hasFocus()) await navigator.clipboard.writeText(text);
      } else if (navigator.clipboard && window.ClipboardItem) {
        await navigator.clipboard.write([new ClipboardItem({ [mime]: new Blob([bytes], { type: mime }) })]);
      }
    } catch (e) { /* clipboard permission denied: the sidebar text box still shows it */ }
  }

  clipboardOut(text) { this.sendText(`cw,${utf8ToB64(text)}`); }

  async upload(files) {
    for (const f of files) {
      const path = f.webkitRelativePath || f.name;
      this.sendText(`FILE_UPLOAD_START:${path}:${f.size}`);
      try {
        for (let off = 0; off < f.size; off += UPLOAD_CHUNK) {
          const chunk = new Uint8Array(await f.slice(off, off + UPLOAD_CHUNK).arrayBuffer());
          const msg = new Uint8Array(chunk.length + 1);
          msg[0] = 0x01;
          msg.set(chunk, 1);
          while (this.ws.bufferedAmount > 8 * UPLOAD_CHUNK) await new Promise((r) => setTimeout(r, 10));
          this.sendBinary(msg);
        }
        this.sendText(`FILE_UPLOAD_END:${path}`);
        this.status(`uploaded ${path}`);
      } catch (e) {
        this.sendText(`FILE_UPLOAD_ERROR:${path}:${e}`);
      }
    }
  }

  // ---------------------------------------------------------------- ui
  status(text) { $('status').textContent = text; }

  renderStats() {
    const s = this.stats;
    const pct = (v) => (v == null ? '-' : `${Math.round(v * 100)}%`);
    const val = (v) => (v == null ? '-' : v);
    $('stats').textContent = [
      `fps ${val(s.fps)}`, `bandwidth ${val(s.mbps)} Mbit/s`, `latency ${val(s.rtt)} ms`,
      `cpu ${val(s.cpu)}%  mem ${pct(s.mem)}`, `gpu ${pct(s.gpu)}  vram ${pct(s.vram)}`,
      `displays ${val(s.displays)}`,
    ].join('\n');
  }

  bindUi() {
    $('toggle').onclick = () => $('sidebar').classList.toggle('open');
    $('encoder').onchange = (e) => this.updateSetting('encoder', e.target.value);
    $('framerate').oninput = (e) => this.updateSetting('framerate', parseInt(e.target.value, 10));
    $('crf').oninput = (e) => this.updateSetting('h264_crf', parseInt(e.target.value, 10));
    $('jpegq').oninput = (e) => this.updateSetting('jpeg_quality', parseInt(e.target.value, 10));
    $('fullcolor').onchange = (e) => this.updateSetting('h264_fullcolor', e.target.checked);
    $('audio').onchange = async (e) => {
      if (e.target.checked) { await this.audio.start(); this.sendText('START_AUDIO'); } else { this.audio.stop(); this.sendText('STOP_AUDIO'); }
    };
    $('mic').onchange = async (e) => {
      if (e.target.checked) await this.audio.startMic((b) => this.sendBinary(b)); else this.audio.stopMic();
    };
    $('video').onchange = (e) => this.sendText(e.target.checked ? 'START_VIDEO' : 'STOP_VIDEO');
    $('fullscreen').onclick = () => document.documentElement.requestFullscreen();
    $('lock').onclick = () => this.input.requestPointerLock();
    $('clip-send').onclick = () => this.clipboardOut($('clip').value);
    $('files').onchange = (e) => this.upload(e.target.files);
    document.addEventListener('dragover', (e) => e.preventDefault());
    document.addEventListener('drop', (e) => { e.preventDefault(); this.upload(e.dataTransfer.files); });
    document.addEventListener('paste', (e) => {
      const text = e.clipboardData && e.clipboardData.getData('text/plain');
      if (text) this.clipboardOut(text);
    });
    let resizeTimer = null;
    window.addEventListener('resize', () => {
      clearTimeout(resizeTimer);
      resizeTimer = setTimeout(() => {
        if (this.settings.is_manual_resolution_mode || this.display.shared) return;
        const dpr = this.settings.use_css_scaling ? 1 : (window.devicePixelRatio || 1);
        this.sendText(`r,${evenDown(window.innerWidth * dpr)}x${evenDown(window.innerHeight * dpr)},${this.display.id}`);
      }, 300);
    });
    document.addEventListener('visibilitychange', () => {
      if (this.display.shared) return;
      this.sendText(document.hidden ? 'STOP_VIDEO' : 'START_VIDEO');
    });
    this.canvas.addEventListener('click', () => { this.canvas.focus(); if (!this.audio.ctx && $('audio').checked) this.audio.start(); });
    window.addEventListener('message', (ev) => {
      if (ev.origin !== window.location.origin) return;   // same-origin embedders / dashboards only
      this.control.handle(ev.data);
    });
    const kbd = $('keyboard-input-assist');
    if (kbd) {
      kbd.addEventListener('compositionstart', () => this.ime.start());
      kbd.addEventListener('compositionend', (e) => { this.ime.end(e.data); kbd.value = ''; });
    }
    this.dashboard = new Dashboard(this);
    this.dashboard.build();
    this.syncUi();
  }
}

const client = new Client();
window.selkiesClient = client;
client.bindUi();
client.connect();
