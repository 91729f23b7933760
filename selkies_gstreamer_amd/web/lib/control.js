// Embedding / dashboard control surface of the client.
//
// * ControlApi: the window.postMessage API the reference dashboards drive
//   (addons/gst-web-core/selkies-core.js receiveMessage, lines 1372-1780): same-origin
//   {type, ...} messages toggle pipelines, resize, change settings, send clipboard and
//   commands; the client answers with sidebarButtonStatusUpdate / stats posts.
// * FallbackPolicy: repeated decoder failures reset the stored settings to safe
//   defaults and reload (selkies-core.js initiateFallback, 4142-4178).
// * SharedProbe: view-only (#shared) clients re-request video (STOP/START_VIDEO, which
//   makes the server send a keyframe) until a video packet arrives (1963-1993).
// * ImeComposer: IME composition text -> keysym press/release messages.
//
// Everything here is DOM-free: the Client passes a `host` with the side effects, so the
// node tests (tests/js/client_test.mjs) drive each message type against a fake host.
import { charToKeysym } from './keysyms.js';

export const SAFE_DEFAULTS = Object.freeze({
  encoder: 'x264enc', h264_fullcolor: false, framerate: 60, h264_crf: 25,
  is_manual_resolution_mode: false, manual_width: 0, manual_height: 0,
});

const evenDown = (v) => Math.max(2, Math.floor(v / 2) * 2);

export class ControlApi {
  // host: { sendText(m), post(obj), shared: bool, displayId: string,
  //         settings: {}, saveSetting(name, value), applySettings(obj),
  //         setManualResolution(w, h), resetResolution(), clearVideo(),
  //         startMic(), stopMic(), audioOn(bool), selectAudioDevice(ctx, id),
  //         setGamepads(bool), setTrackpad(bool), setSynth(v), showKeyboard(),
  //         fullscreen(), setClipboard(text), statsSnapshot(), updateRendering() }
  constructor(host) {
    this.host = host;
    this.state = { video: true, audio: false, microphone: false, gamepad: true };
    this.sidebarOpen = false;
  }

  statusUpdate() {
    this.host.post({ type: 'sidebarButtonStatusUpdate', ...this.state });
  }

  // Returns true when the message was understood (dispatched or deliberately ignored
  // for this client role), false for malformed / unknown messages.
  handle(msg) {
    const h = this.host;
    if (typeof msg !== 'object' || msg === null || typeof msg.type !== 'string') return false;
    const shared = !!h.shared;
    const bool = (name) => {
      if (typeof msg.value !== 'boolean') return false;
      h.saveSetting(name, msg.value);
      return true;
    };
    switch (msg.type) {
      case 'sidebarVisibilityChanged': this.sidebarOpen = !!msg.isOpen; return true;
      case 'setScaleLocally': return shared ? true : bool('scale_locally');
      case 'setUseCssScaling':
        if (!bool('use_css_scaling')) return false;
        h.updateRendering();
        if (!shared) h.applySettings({});   // resolution follows the new pixel ratio
        return true;
      case 'setAntiAliasing': if (!bool('anti_aliasing')) return false; h.updateRendering(); return true;
      case 'setUseBrowserCursors': if (!bool('use_browser_cursors')) return false; h.updateRendering(); return true;
      case 'setSynth': h.setSynth(msg.value); return true;
      case 'showVirtualKeyboard': if (!shared) h.showKeyboard(); return true;
      case 'setManualResolution': {
        if (shared) return true;
        const w = parseInt(msg.width, 10), hh = parseInt(msg.height, 10);
        if (!(w > 0) || !(hh > 0)) return false;
        h.setManualResolution(evenDown(w), evenDown(hh));
        return true;
      }
      case 'resetResolutionToWindow': if (!shared) h.resetResolution(); return true;
      case 'settings':
        if (typeof msg.settings !== 'object' || msg.settings === null) return false;
        if (!shared) h.applySettings(msg.settings);
        return true;
      case 'getStats': h.post({ type: 'stats', data: h.statsSnapshot() }); return true;
      case 'clipboardUpdateFromUI':
        if (typeof msg.text !== 'string') return false;
        if (!shared) h.setClipboard(msg.text);
        return true;
      case 'pipelineStatusUpdate': {
        let changed = false;
        for (const k of ['video', 'audio', 'microphone', 'gamepad']) {
          if (msg[k] !== undefined && this.state[k] !== !!msg[k]) { this.state[k] = !!msg[k]; changed = true; }
        }
        if (changed) this.statusUpdate();
        return true;
      }
      case 'pipelineControl': return this._pipeline(msg.pipeline, !!msg.enabled);
      case 'audioDeviceSelected':
        if (!msg.deviceId || (msg.context !== 'input' && msg.context !== 'output')) return false;
        if (shared && msg.context === 'input') return true;
        h.selectAudioDevice(msg.context, msg.deviceId);
        return true;
      case 'gamepadControl': {
        const on = !!msg.enabled;
        if (this.state.gamepad !== on) {
          this.state.gamepad = on;
          h.saveSetting('gamepad_enabled', on);
          h.setGamepads(shared || on);   // view-only clients keep their pads (player links)
          this.statusUpdate();
        }
        return true;
      }
      case 'requestFullscreen': h.fullscreen(); return true;
      case 'command':
        if (typeof msg.value !== 'string') return false;
        if (!shared) h.sendText(`cmd,${msg.value}`);
        return true;
      case 'touchinput:trackpad':
      case 'touchinput:touch': {
        const tp = msg.type === 'touchinput:trackpad';
        h.saveSetting('trackpad_mode', tp);
        h.setTrackpad(tp);
        h.sendText(`SET_NATIVE_CURSOR_RENDERING,${tp ? 1 : 0}`);
        return true;
      }
      default: return false;
    }
  }

  _pipeline(name, on) {
    const h = this.host;
    if (name === 'video') {
      if (h.shared) return true;
      if (this.state.video === on) return true;
      this.state.video = on;
      h.clearVideo();
      h.sendText(on ? 'START_VIDEO' : 'STOP_VIDEO');
    } else if (name === 'audio') {
      if (h.displayId !== 'primary') return true;   // audio belongs to the primary display
      if (this.state.audio === on) return true;
      this.state.audio = on;
      h.audioOn(on);
      h.sendText(on ? 'START_AUDIO' : 'STOP_AUDIO');
    } else if (name === 'microphone') {
      if (h.shared) return true;
      if (this.state.microphone === on) return true;
      this.state.microphone = on;
      if (on) h.startMic(); else h.stopMic();
    } else {
      return false;
    }
    this.statusUpdate();
    return true;
  }
}

// Decoder failures: one error may be a transient (a stripe decoder closed mid-resize);
// `limit` errors within `windowMs` mean this browser cannot decode the stream as
// configured. Then: shared clients just reload (they follow the primary's settings);
// others store SAFE_DEFAULTS first (full-frame H.264, 4:2:0) so the reload starts from
// a configuration every WebCodecs implementation decodes.
export class FallbackPolicy {
  constructor(limit = 3, windowMs = 10000) {
    this.limit = limit;
    this.windowMs = windowMs;
    this.times = [];
    this.triggered = false;
  }

  // -> null (keep going) or {resetSettings: bool, reloadAfterMs}
  onError(nowMs, shared) {
    if (this.triggered) return null;
    this.times = this.times.filter((t) => nowMs - t < this.windowMs);
    this.times.push(nowMs);
    if (this.times.length < this.limit) return null;
    this.triggered = true;
    return { resetSettings: !shared, reloadAfterMs: 3000 };
  }
}

// #shared viewers: after connecting, and whenever `timeoutMs` passes without a video
// packet, ask the server for a fresh keyframe by cycling STOP_VIDEO / START_VIDEO;
// give up after `maxAttempts`.
export class SharedProbe {
  constructor(timeoutMs = 4000, maxAttempts = 5) {
    this.timeoutMs = timeoutMs;
    this.maxAttempts = maxAttempts;
    this.reset(0);
  }

  reset(nowMs) {
    this.state = 'awaiting';
    this.attempts = 0;
    this.deadline = nowMs + this.timeoutMs;
  }

  onVideo() { this.state = 'streaming'; }

  // -> list of text messages to send now ([] when nothing to do); state 'error' at the end
  tick(nowMs) {
    if (this.state !== 'awaiting' || nowMs < this.deadline) return [];
    this.attempts++;
    if (this.attempts >= this.maxAttempts) { this.state = 'error'; return []; }
    this.deadline = nowMs + this.timeoutMs;
    return ['STOP_VIDEO', 'START_VIDEO'];
  }
}

// IME composition (compositionstart/update/end on the focused assist input): keydown
// events during composition carry no final text (isComposing), so nothing is sent until
// compositionend, whose text is typed out as keysym press/release pairs.
export class ImeComposer {
  constructor(send) {
    this.send = send;
    this.composing = false;
  }

  start() { this.composing = true; }

  end(text) {
    this.composing = false;
    if (!text) return 0;
    let n = 0;
    for (const ch of text) {
      const ks = charToKeysym(ch);
      if (ks == null) continue;
      this.send(`kd,${ks}`);
      this.send(`ku,${ks}`);
      n++;
    }
    return n;
  }
}
