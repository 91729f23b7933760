// Stripe video renderer: one WebCodecs VideoDecoder per H.264 stripe (0x04)
// and createImageBitmap for JPEG stripes (0x03), composited onto one canvas.
// Full-frame H.264 arrives as a single stripe at y = 0.

export class VideoRenderer {
  constructor(canvas, onError) {
    this.canvas = canvas;
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
    if (info && info.decoder.state !== 'closed' && info.width === width && info.height === height) return info;
    if (info) {
      try { info.decoder.close(); } catch (e) { /* ignore */ }
    }
    const decoder = new VideoDecoder({
      output: (frame) => this._paint(frame, y),
      error: (e) => { this.decoders.delete(y); this.onError(e); },
    });
    decoder.configure({ codec: 'avc1.42E01E', codedWidth: width, codedHeight: height, optimizeForLatency: true });
    info = { decoder, width, height, keyed: false };
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

  h264(pkt) {
    this.frameIds.add(pkt.frameId);
    this.lastFrameId = pkt.frameId;
    if (typeof VideoDecoder === 'undefined') return;
    const info = this._decoderFor(pkt.y, pkt.width, pkt.height);
    if (!pkt.key && !info.keyed) return;   // wait for this stripe's IDR
    if (pkt.key) info.keyed = true;
    if (info.decoder.decodeQueueSize > 30) return;  // decoder falling behind: drop deltas until next key
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
