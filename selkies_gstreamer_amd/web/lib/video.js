// Stripe video renderer: one WebCodecs VideoDecoder per H.264 stripe (0x04)
// and createImageBitmap for JPEG stripes (0x03), composited onto one canvas.
// Full-frame H.264 arrives as a single stripe at y = 0; so do the HEVC (x265enc,
// Annex B with in-band parameter sets) and AV1 (svtav1enc, OBU temporal units) frames
// of the MI355X encoders, which use the same 0x04 framing.

// Level tables of the encoders (csrc/codec/hevc_params.cpp choose_level_idc,
// csrc/codec/av1_cpu.cpp choose_level_idx): the codec string names the stream's level.
const HEVC_LEVELS = [[30, 36864, 552960], [60, 122880, 3686400], [63, 245760, 7372800], [90, 552960, 16588800],
  [93, 983040, 33177600], [120, 2228224, 66846720], [123, 2228224, 133693440], [150, 8912896, 267386880],
  [153, 8912896, 534773760], [156, 8912896, 1069547520], [180, 35651584, 1069547520],
  [183, 35651584, 2139095040], [186, 35651584, 4278190080]];
const AV1_LEVELS = [[0, 147456, 4423680], [1, 278784, 8363520], [4, 665856, 19975680], [5, 1065024, 31950720],
  [8, 2359296, 70778880], [9, 2359296, 141557760], [12, 8912896, 267386880], [13, 8912896, 534773760],
  [14, 8912896, 1069547520], [16, 35651584, 1069547520], [17, 35651584, 2139095040],
  [18, 35651584, 4278190080]];
function pickLevel(table, w, h, fps, dflt) {
  const ps = w * h, sr = ps * (fps > 0 ? fps : 60);
  for (const [lv, mps, msr] of table) if (ps <= mps && sr <= msr) return lv;
  return dflt;
}
// WebCodecs codec string of the negotiated encoder for a w x h stream at fps (coded
// size: HEVC pads to 16, the level limits use it).
export function codecString(encoder, w, h, fps = 60) {
  if (encoder === 'x265enc') {
    const pw = (w + 15) & ~15, ph = (h + 15) & ~15;
    return `hev1.1.6.L${pickLevel(HEVC_LEVELS, pw, ph, fps, 186)}.B0`;
  }
  if (encoder === 'svtav1enc') {
    const idx = pickLevel(AV1_LEVELS, w, h, fps, 31);
    return `av01.0.${String(idx).padStart(2, '0')}M.08`;
  }
  return 'avc1.42E01E';
}

// Least time between two key-frame requests of one stripe (REQUEST_KEYFRAME).
export const KEY_REQUEST_INTERVAL_MS = 250;

export class VideoRenderer {
  // onKeyframeNeeded(y): the stripe at y cannot decode deltas any more (a chunk was dropped,
  // or its decoder was recreated) and needs a key frame; the client sends REQUEST_KEYFRAME.
  constructor(canvas, onError, onKeyframeNeeded) {
    this.canvas = canvas;
    this.onKeyframeNeeded = onKeyframeNeeded || (() => {});
    this.keyRequestedAt = new Map();   // y -> time of the last request
    this.dropped = 0;                  // delta chunks dropped because the decoder fell behind
    this.encoder = 'x264enc';   // set from the negotiated settings (codecString)
    this.fps = 60;
    this.ctx = canvas.getContext('2d', { alpha: false, desynchronized: true });
    this.decoders = new Map();   // y -> {decoder, width, height, keyed}
    this.onError = onError || ((e) => console.error(e));
    this.framesPainted = 0;
    this.frameIds = new Set();
    this.lastFrameId = -1;
  }

  resize(w, h) {
    if (this.canvas.width !== w || this.canvas.height !== h) {
      this.canvas.width = w;
      this.canvas.height = h;
      this.ctx.fillStyle = '#000';
      this.ctx.fillRect(0, 0, w, h);
    }
  }

  reset() {
    for (const info of this.decoders.values()) {
      try { if (info.decoder.state !== 'closed') info.decoder.close(); } catch (e) { /* ignore */ }
    }
    this.decoders.clear();
  }

  _decoderFor(y, width, height) {
    let info = this.decoders.get(y);
    const codec = codecString(this.encoder, width, height, this.fps);
    if (info && info.decoder.state !== 'closed' && info.width === width && info.height === height &&
        info.codec === codec) return info;
    if (info) {
      try { info.decoder.close(); } catch (e) { /* ignore */ }
    }
    const decoder = new VideoDecoder({
      output: (frame) => this._paint(frame, y),
      error: (e) => { this.decoders.delete(y); this.onError(e); },
    });
    const cfg = { codec, codedWidth: width, codedHeight: height, optimizeForLatency: true };
    if (codec.startsWith('hev1')) cfg.hevc = { format: 'annexb' };
    decoder.configure(cfg);
    info = { decoder, width, height, keyed: false, codec };
    this.decoders.set(y, info);
    return info;
  }

  _paint(frame, y) {
    try {
      this.ctx.drawImage(frame, 0, y, frame.displayWidth, frame.displayHeight);
      this.framesPainted++;
    } finally {
      frame.close();
    }
  }

  _requestKey(y) {
    const now = performance.now();
    const last = this.keyRequestedAt.get(y);
    if (last !== undefined && now - last < KEY_REQUEST_INTERVAL_MS) return;
    this.keyRequestedAt.set(y, now);
    this.onKeyframeNeeded(y);
  }

  h264(pkt) {
    this.frameIds.add(pkt.frameId);
    this.lastFrameId = pkt.frameId;
    if (typeof VideoDecoder === 'undefined') return;
    const info = this._decoderFor(pkt.y, pkt.width, pkt.height);
    if (!pkt.key && !info.keyed) {   // no reference for this delta: wait for the stripe's key frame
      this._requestKey(pkt.y);        // (the default GOP is infinite: ask for one)
      return;
    }
    if (pkt.key) {
      info.keyed = true;
      this.keyRequestedAt.delete(pkt.y);
    }
    if (!pkt.key && info.decoder.decodeQueueSize > 30) {
      // the decoder fell behind: drop this delta, and with it every delta up to the next
      // key frame (they predict from the dropped one), which is requested now
      info.keyed = false;
      this.dropped++;
      this._requestKey(pkt.y);
      return;
    }
    info.decoder.decode(new EncodedVideoChunk({
      type: pkt.key ? 'key' : 'delta', timestamp: performance.now() * 1000, data: pkt.payload,
    }));
  }

  async jpeg(pkt) {
    this.frameIds.add(pkt.frameId);
    this.lastFrameId = pkt.frameId;
    const bmp = await createImageBitmap(new Blob([pkt.payload], { type: 'image/jpeg' }));
    this.ctx.drawImage(bmp, 0, pkt.y);
    bmp.close();
    this.framesPainted++;
  }

  takeFps(elapsedMs) {
    const fps = elapsedMs > 0 ? (this.frameIds.size * 1000) / elapsedMs : 0;
    this.frameIds.clear();
    return fps;
  }
}
