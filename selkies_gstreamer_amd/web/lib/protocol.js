// Wire protocol helpers shared by the client modules (pure functions, unit
// tested under node: tests/js/client_test.mjs). Server side: server/protocol.py.

export const PKT_AUDIO = 0x01;
export const PKT_JPEG = 0x03;
export const PKT_H264 = 0x04;

// Parses a binary server frame. Returns null for unknown / short frames.
//  0x01 0x00 opus...                                  -> {type:'audio', payload}
//  0x03 0x00 fid16 y16 jpeg...                        -> {type:'jpeg', frameId, y, payload}
//  0x04 key fid16 y16 w16 h16 annexb...               -> {type:'h264', key, frameId, y, width, height, payload}
export function parseFrame(buf) {
  const u8 = buf instanceof Uint8Array ? buf : new Uint8Array(buf);
  if (u8.length < 2) return null;
  const dv = new DataView(u8.buffer, u8.byteOffset, u8.byteLength);
  switch (u8[0]) {
    case PKT_AUDIO:
      return { type: 'audio', payload: u8.subarray(2) };
    case PKT_JPEG:
      if (u8.length < 6) return null;
      return { type: 'jpeg', frameId: dv.getUint16(2, false), y: dv.getUint16(4, false), payload: u8.subarray(6) };
    case PKT_H264:
      if (u8.length < 10) return null;
      return {
        type: 'h264', key: u8[1] === 1, frameId: dv.getUint16(2, false), y: dv.getUint16(4, false),
        width: dv.getUint16(6, false), height: dv.getUint16(8, false), payload: u8.subarray(10),
      };
    default:
      return null;
  }
}

// Text control messages -> {kind, ...}
export function parseText(msg) {
  if (msg.startsWith('{')) {
    try { return { kind: 'json', data: JSON.parse(msg) }; } catch (e) { return { kind: 'unknown', msg }; }
  }
  const word = (p) => msg.startsWith(p);
  if (word('MODE ')) return { kind: 'mode', mode: msg.slice(5) };
  if (word('KILL')) return { kind: 'kill', reason: msg.slice(5) };
  if (word('PIPELINE_RESETTING')) return { kind: 'reset', display: msg.split(' ')[1] || 'primary' };
  if (word('DISPLAY_CONFIG_UPDATE,')) return { kind: 'displays', data: JSON.parse(msg.slice(22)) };
  if (word('cursor,')) return { kind: 'cursor', data: JSON.parse(msg.slice(7)) };
  if (word('clipboard_binary,')) {
    const rest = msg.slice(17);
    const i = rest.indexOf(',');
    return { kind: 'clipboard', mime: rest.slice(0, i), b64: rest.slice(i + 1) };
  }
  if (word('clipboard,')) return { kind: 'clipboard', mime: 'text/plain', b64: msg.slice(10) };
  if (word('clipboard_start,')) {
    const [, mime, size] = msg.split(',');
    return { kind: 'clipboard_start', mime, size: parseInt(size, 10) };
  }
  if (word('clipboard_data,')) return { kind: 'clipboard_data', b64: msg.slice(15) };
  if (msg === 'clipboard_finish') return { kind: 'clipboard_finish' };
  if (['VIDEO_STARTED', 'VIDEO_STOPPED', 'AUDIO_STARTED', 'AUDIO_STOPPED'].includes(msg)) return { kind: 'state', msg };
  return { kind: 'unknown', msg };
}

// Mouse button mask bits used by the server (server/input.py).
export const MASK_LEFT = 1, MASK_MIDDLE = 2, MASK_RIGHT = 4, MASK_WHEEL_DOWN = 8, MASK_WHEEL_UP = 16;
export const MASK_WHEEL_LEFT = 64, MASK_WHEEL_RIGHT = 128;
export function buttonBit(domButton) {
  // DOM: 0 left, 1 middle, 2 right, 3 back, 4 forward  -> bits 0..4
  return domButton >= 0 && domButton <= 4 ? (1 << domButton) : 0;
}

export function mouseMessage(relative, x, y, mask, magnitude = 0) {
  return `${relative ? 'm2' : 'm'},${Math.round(x)},${Math.round(y)},${mask},${magnitude}`;
}

// Maps a client pixel position on an element of size (cw, ch) to stream
// coordinates of a (sw, sh) stream drawn with letterboxing (object-fit: contain).
export function toStreamCoords(px, py, cw, ch, sw, sh) {
  if (!sw || !sh || !cw || !ch) return [0, 0];
  const scale = Math.min(cw / sw, ch / sh);
  const ox = (cw - sw * scale) / 2, oy = (ch - sh * scale) / 2;
  const x = Math.min(sw - 1, Math.max(0, (px - ox) / scale));
  const y = Math.min(sh - 1, Math.max(0, (py - oy) / scale));
  return [Math.round(x), Math.round(y)];
}

export function evenDown(v) { return Math.max(2, Math.floor(v) & ~1); }

export function b64encode(bytes) {
  let s = '';
  for (let i = 0; i < bytes.length; i += 0x8000) s += String.fromCharCode.apply(null, bytes.subarray(i, i + 0x8000));
  return btoa(s);
}

export function b64decode(b64) {
  const s = atob(b64);
  const out = new Uint8Array(s.length);
  for (let i = 0; i < s.length; i++) out[i] = s.charCodeAt(i);
  return out;
}

export function utf8ToB64(text) { return b64encode(new TextEncoder().encode(text)); }
export function b64ToUtf8(b64) { return new TextDecoder().decode(b64decode(b64)); }

// Float32 mono/stereo PCM at `inRate` -> s16le mono at 24 kHz (microphone uplink).
export function downsampleToS16Mono(channels, inRate, outRate = 24000) {
  const n = channels[0].length;
  const ratio = inRate / outRate;
  const outLen = Math.floor(n / ratio);
  const out = new Int16Array(outLen);
  for (let i = 0; i < outLen; i++) {
    const start = Math.floor(i * ratio), end = Math.min(n, Math.floor((i + 1) * ratio));
    let acc = 0, cnt = 0;
    for (let j = start; j < Math.max(end, start + 1) && j < n; j++) {
      let v = 0;
      for (const ch of channels) v += ch[j];
      acc += v / channels.length;
      cnt++;
    }
    const s = Math.max(-1, Math.min(1, cnt ? acc / cnt : 0));
    out[i] = s < 0 ? s * 0x8000 : s * 0x7fff;
  }
  return out;
}
