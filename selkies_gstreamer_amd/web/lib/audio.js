// Audio: Opus packets (0x01) -> WebCodecs AudioDecoder -> AudioWorklet ring
// buffer; microphone -> AudioWorklet capture -> s16le mono 24 kHz (0x02).
import { downsampleToS16Mono } from './protocol.js';

const PLAYER = `
class SelkiesPlayer extends AudioWorkletProcessor {
  constructor() {
    super();
    this.q = []; this.off = 0; this.buffered = 0;
    this.port.onmessage = (e) => { this.q.push(e.data); this.buffered += e.data[0].length;
      while (this.buffered > sampleRate * 0.25) { const d = this.q.shift(); this.buffered -= d[0].length; this.off = 0; } };
  }
  process(inputs, outputs) {
    const out = outputs[0];
    for (let i = 0; i < out[0].length; i++) {
      if (!this.q.length) { for (const ch of out) ch[i] = 0; continue; }
      const cur = this.q[0];
      for (let c = 0; c < out.length; c++) out[c][i] = cur[Math.min(c, cur.length - 1)][this.off];
      if (++this.off >= cur[0].length) { this.q.shift(); this.buffered -= cur[0].length; this.off = 0; }
    }
    return true;
  }
}
registerProcessor('selkies-player', SelkiesPlayer);
class SelkiesMic extends AudioWorkletProcessor {
  process(inputs) {
    const inp = inputs[0];
    if (inp && inp.length) this.port.postMessage(inp.map((c) => c.slice(0)));
    return true;
  }
}
registerProcessor('selkies-mic', SelkiesMic);
`;

export class AudioPipeline {
  constructor() {
    this.ctx = null;
    this.node = null;
    this.decoder = null;
    this.micStream = null;
    this.micNode = null;
    this.enabled = false;
  }

  async start() {
    if (this.ctx) { await this.ctx.resume(); this.enabled = true; return; }
    if (typeof AudioDecoder === 'undefined') return;
    this.ctx = new AudioContext({ sampleRate: 48000, latencyHint: 'interactive' });
    const url = URL.createObjectURL(new Blob([PLAYER], { type: 'application/javascript' }));
    await this.ctx.audioWorklet.addModule(url);
    this.node = new AudioWorkletNode(this.ctx, 'selkies-player', { outputChannelCount: [2] });
    this.node.connect(this.ctx.destination);
    this.decoder = new AudioDecoder({
      output: (data) => {
        const chans = [];
        for (let c = 0; c < data.numberOfChannels; c++) {
          const buf = new Float32Array(data.numberOfFrames);
          data.copyTo(buf, { planeIndex: c, format: 'f32-planar' });
          chans.push(buf);
        }
        data.close();
        this.node.port.postMessage(chans);
      },
      error: (e) => console.warn('audio decoder', e),
    });
    this.decoder.configure({ codec: 'opus', sampleRate: 48000, numberOfChannels: 2 });
    this.enabled = true;
  }

  stop() {
    this.enabled = false;
    if (this.ctx) this.ctx.suspend();
  }

  opus(payload) {
    if (!this.enabled || !this.decoder || this.decoder.state !== 'configured') return;
    this.decoder.decode(new EncodedAudioChunk({ type: 'key', timestamp: performance.now() * 1000, data: payload }));
  }

  async startMic(send) {
    if (!this.ctx) await this.start();
    if (!this.ctx || this.micNode) return;
    this.micStream = await navigator.mediaDevices.getUserMedia({
      audio: { echoCancellation: true, noiseSuppression: true, channelCount: 1 },
    });
    const src = this.ctx.createMediaStreamSource(this.micStream);
    this.micNode = new AudioWorkletNode(this.ctx, 'selkies-mic');
    let pending = [], count = 0;
    this.micNode.port.onmessage = (e) => {
      const pcm = downsampleToS16Mono(e.data, this.ctx.sampleRate, 24000);
      pending.push(pcm);
      count += pcm.length;
      if (count < 480) return;   // ~20 ms per uplink message
      const out = new Uint8Array(1 + 2 * count);
      out[0] = 0x02;
      let o = 1;
      for (const p of pending) { out.set(new Uint8Array(p.buffer), o); o += p.byteLength; }
      pending = [];
      count = 0;
      send(out);
    };
    src.connect(this.micNode);
  }

  stopMic() {
    if (this.micStream) this.micStream.getTracks().forEach((t) => t.stop());
    if (this.micNode) this.micNode.disconnect();
    this.micStream = null;
    this.micNode = null;
  }
}
