// Unit tests of the browser client's pure modules (run by tests/test_web_client.py).
import assertModule from 'assert';
const assert = assertModule.strict;
import * as dash from '../../selkies_gstreamer_amd/web/lib/dashboard.js';
import {
  ControlApi, FallbackPolicy, SharedProbe, ImeComposer, SAFE_DEFAULTS,
} from '../../selkies_gstreamer_amd/web/lib/control.js';
import * as tg from '../../selkies_gstreamer_amd/web/lib/touch-gamepad.js';
// node < 16 has no btoa/atob (browsers do)
if (typeof globalThis.btoa === 'undefined') {
  globalThis.btoa = (s) => Buffer.from(s, 'binary').toString('base64');
  globalThis.atob = (b) => Buffer.from(b, 'base64').toString('binary');
}
import { keysymFor, charToKeysym } from '../../selkies_gstreamer_amd/web/lib/keysyms.js';
import {
  parseFrame, parseText, toStreamCoords, mouseMessage, buttonBit, downsampleToS16Mono, utf8ToB64, b64ToUtf8, evenDown,
} from '../../selkies_gstreamer_amd/web/lib/protocol.js';

// keysyms
assert.equal(keysymFor({ key: 'a', code: 'KeyA' }), 0x61);
assert.equal(keysymFor({ key: 'A', code: 'KeyA' }), 0x41);
assert.equal(keysymFor({ key: 'Enter', code: 'Enter' }), 0xff0d);
assert.equal(keysymFor({ key: 'Enter', code: 'NumpadEnter' }), 0xff8d);
assert.equal(keysymFor({ key: 'Shift', code: 'ShiftRight' }), 0xffe2);
assert.equal(keysymFor({ key: 'Control', code: 'ControlLeft' }), 0xffe3);
assert.equal(keysymFor({ key: 'F12', code: 'F12' }), 0xffc9);
assert.equal(keysymFor({ key: '€', code: 'KeyE' }), 0x010020ac);
assert.equal(keysymFor({ key: 'é', code: 'Digit2' }), 0xe9);
assert.equal(keysymFor({ key: 'Dead', code: 'BracketLeft' }), null);
assert.equal(keysymFor({ key: '1', code: 'Numpad1', getModifierState: () => true }), 0xffb1);
assert.equal(keysymFor({ key: 'End', code: 'Numpad1', getModifierState: () => false }), 0xff9c);
assert.equal(charToKeysym('😀'), (0x01000000 | 0x1f600) >>> 0);

// binary frames
const h264 = new Uint8Array([0x04, 1, 0x12, 0x34, 0, 64, 7, 128, 0, 64, 0, 0, 0, 1, 0x67]);
const f = parseFrame(h264.buffer);
assert.deepEqual([f.type, f.key, f.frameId, f.y, f.width, f.height, f.payload.length], ['h264', true, 0x1234, 64, 1920, 64, 5]);
const jpeg = parseFrame(new Uint8Array([0x03, 0, 0, 7, 0, 128, 0xff, 0xd8]));
assert.deepEqual([jpeg.type, jpeg.frameId, jpeg.y, jpeg.payload[0]], ['jpeg', 7, 128, 0xff]);
assert.equal(parseFrame(new Uint8Array([0x01, 0, 9, 9])).payload.length, 2);
assert.equal(parseFrame(new Uint8Array([0x09, 0])), null);

// text messages
assert.deepEqual(parseText('MODE websockets'), { kind: 'mode', mode: 'websockets' });
assert.equal(parseText('KILL a new primary client connected connection killed').kind, 'kill');
assert.deepEqual(parseText('PIPELINE_RESETTING display2'), { kind: 'reset', display: 'display2' });
assert.deepEqual(parseText('DISPLAY_CONFIG_UPDATE,{"type":"display_config_update","displays":["primary"]}').data.displays, ['primary']);
assert.equal(parseText('cursor,{"curdata":"","handle":3}').data.handle, 3);
assert.deepEqual(parseText('clipboard_binary,image/png,AAEC'), { kind: 'clipboard', mime: 'image/png', b64: 'AAEC' });
assert.equal(b64ToUtf8(parseText('clipboard,' + utf8ToB64('héllo')).b64), 'héllo');
assert.deepEqual(parseText('clipboard_start,text/plain,5'), { kind: 'clipboard_start', mime: 'text/plain', size: 5 });
assert.equal(parseText('{"type":"stream_resolution","width":2,"height":4}').data.width, 2);

// pointer
assert.deepEqual(toStreamCoords(50, 50, 100, 100, 200, 200), [100, 100]);
assert.deepEqual(toStreamCoords(0, 25, 200, 100, 100, 100), [0, 25]);     // left of the letterboxed image
assert.deepEqual(toStreamCoords(150, 50, 200, 100, 100, 100), [99, 50]);  // clamp
assert.equal(mouseMessage(false, 10.4, 20.6, 1), 'm,10,21,1,0');
assert.equal(mouseMessage(true, -3, 4, 0, 2), 'm2,-3,4,0,2');
assert.deepEqual([0, 1, 2, 3, 4, 5].map(buttonBit), [1, 2, 4, 8, 16, 0]);
assert.equal(evenDown(1921.5), 1920);

// microphone downsampling 48k -> 24k s16 mono
const a = new Float32Array(480).fill(0.5), b = new Float32Array(480).fill(-0.5);
const pcm = downsampleToS16Mono([a, a], 48000);
assert.equal(pcm.length, 240);
assert.equal(pcm[0], Math.trunc(0.5 * 0x7fff));
assert.equal(downsampleToS16Mono([a, b], 48000)[10], 0);

// ---- dashboard helpers (lib/dashboard.js) and the touch gamepad (lib/touch-gamepad.js)
{
  const all = dash.visibleSections({});
  assert.ok(all.has('video') && all.has('sharing') && all.has('softkeys'));
  const some = dash.visibleSections({ ui_sidebar_show_stats: { value: false }, command_enabled: { value: false },
    file_transfers: { value: 'download' } });
  assert.ok(!some.has('stats') && !some.has('apps') && !some.has('files') && some.has('video'));
  assert.equal(dash.visibleSections({ ui_show_sidebar: { value: false } }).size, 0);
  const links = dash.sharingLinks('http://h:8082/index.html#x', { enable_player3: { value: false } });
  assert.deepEqual(links.map((l) => l.url), ['http://h:8082/index.html#shared', 'http://h:8082/index.html#player2',
    'http://h:8082/index.html#player4']);
  assert.deepEqual(dash.sharingLinks('http://h/', { enable_sharing: { value: false } }), []);
  assert.deepEqual(dash.parseRole('#player3'), { id: 'primary', position: 'right', shared: true, player: 3 });
  assert.equal(dash.parseRole('#shared').player, 0);
  assert.equal(dash.parseRole('#display2-left').position, 'left');
  assert.deepEqual(dash.softKeyMessages('Ctrl+Alt+Del'),
    ['kd,65507', 'kd,65513', 'kd,65535', 'ku,65535', 'ku,65513', 'ku,65507']);
  const r = new dash.Ring(4);
  [1, 2, 3, 4, 5].forEach((x) => r.push(x));
  assert.deepEqual(r.v, [2, 3, 4, 5]);
  const pts = dash.sparkPoints(r, 4, 10);
  assert.equal(pts.length, 4);
  assert.equal(pts[3][1], 1);          // max at the top (y = 1)

  assert.deepEqual(tg.stickAxes(0, 0, 50), [0, 0]);
  assert.deepEqual(tg.stickAxes(5, 0, 50), [0, 0]);       // inside the dead zone
  assert.deepEqual(tg.stickAxes(100, 0, 50), [1, 0]);     // clamped to the unit circle
  const [sx, sy] = tg.stickAxes(30, -30, 50);
  assert.ok(sx > 0.4 && sy < -0.4 && Math.hypot(sx, sy) <= 1);
  assert.deepEqual(tg.dpadButtons(10, 0), [tg.BUTTONS.RIGHT]);
  assert.deepEqual(tg.dpadButtons(10, 10).sort(), [tg.BUTTONS.DOWN, tg.BUTTONS.RIGHT].sort());
  assert.deepEqual(tg.dpadButtons(0, -10), [tg.BUTTONS.UP]);
  assert.deepEqual(tg.dpadButtons(0.01, 0.01), []);
  const pad = new tg.VirtualPad(1);
  assert.equal(pad.buttons.length, 17);
  assert.ok(pad.setButton(tg.BUTTONS.A, true));
  assert.ok(!pad.setButton(tg.BUTTONS.A, true));          // no change
  pad.setStick('right', 0.5, -0.5);
  assert.deepEqual(pad.axes, [0, 0, 0.5, -0.5]);
  const nav = { getGamepads: () => [{ index: 0, id: 'real' }] };
  assert.equal(tg.freeIndex(nav), 1);
  const undo = tg.installGetGamepads(nav, pad);
  assert.equal(nav.getGamepads()[1], pad);
  undo();
  assert.equal(nav.getGamepads().length, 1);
}

// ---------------------------------------------------------------- postMessage control API
{
  const mkHost = (over = {}) => {
    const h = { sent: [], posted: [], calls: [], saved: {}, shared: false, displayId: 'primary' };
    const rec = (name) => (...a) => h.calls.push([name, ...a]);
    Object.assign(h, {
      sendText: (m) => h.sent.push(m), post: (o) => h.posted.push(o),
      saveSetting: (k, v) => { h.saved[k] = v; }, applySettings: rec('applySettings'),
      setManualResolution: (w, hh) => { h.calls.push(['res', w, hh]); h.sent.push(`r,${w}x${hh},primary`); },
      resetResolution: rec('resetResolution'), clearVideo: rec('clearVideo'), startMic: rec('startMic'),
      stopMic: rec('stopMic'), audioOn: rec('audioOn'), selectAudioDevice: rec('selectAudioDevice'),
      setGamepads: rec('setGamepads'), setTrackpad: rec('setTrackpad'), setSynth: rec('setSynth'),
      showKeyboard: rec('showKeyboard'), fullscreen: rec('fullscreen'), setClipboard: rec('setClipboard'),
      statsSnapshot: () => ({ fps: 60 }), updateRendering: rec('updateRendering'),
    }, over);
    return h;
  };
  const h = mkHost();
  const c = new ControlApi(h);
  // every reference message type is understood
  const all = [
    { type: 'sidebarVisibilityChanged', isOpen: true }, { type: 'setScaleLocally', value: true },
    { type: 'setSynth', value: 'x' }, { type: 'showVirtualKeyboard' }, { type: 'setUseCssScaling', value: true },
    { type: 'setAntiAliasing', value: false }, { type: 'setUseBrowserCursors', value: true },
    { type: 'setManualResolution', width: 1281, height: 721 }, { type: 'resetResolutionToWindow' },
    { type: 'settings', settings: { framerate: 30 } }, { type: 'getStats' },
    { type: 'clipboardUpdateFromUI', text: 'hi' }, { type: 'pipelineStatusUpdate', audio: true },
    { type: 'pipelineControl', pipeline: 'video', enabled: false },
    { type: 'audioDeviceSelected', context: 'output', deviceId: 'spk' }, { type: 'gamepadControl', enabled: false },
    { type: 'requestFullscreen' }, { type: 'command', value: 'xterm' }, { type: 'touchinput:trackpad' },
    { type: 'touchinput:touch' },
  ];
  for (const m of all) assert.equal(c.handle(m), true, m.type);
  assert.equal(c.handle({ type: 'nope' }), false);
  assert.equal(c.handle(null), false);
  assert.equal(c.handle({ type: 'setManualResolution', width: 'x', height: 5 }), false);
  // the WebSocket messages the reference sends for them
  assert.deepEqual(h.sent, ['r,1280x720,primary', 'STOP_VIDEO', 'cmd,xterm', 'SET_NATIVE_CURSOR_RENDERING,1',
    'SET_NATIVE_CURSOR_RENDERING,0']);
  assert.deepEqual(h.posted.find((p) => p.type === 'stats'), { type: 'stats', data: { fps: 60 } });
  const upd = h.posted.filter((p) => p.type === 'sidebarButtonStatusUpdate');
  assert.equal(upd.length, 3);   // audio status, video off, gamepad off
  assert.deepEqual(upd[2], { type: 'sidebarButtonStatusUpdate', video: false, audio: true, microphone: false, gamepad: false });
  assert.equal(h.saved.use_css_scaling, true);
  assert.equal(h.saved.anti_aliasing, false);
  assert.deepEqual(h.calls.find((x) => x[0] === 'applySettings' && x[1].framerate), ['applySettings', { framerate: 30 }]);
  // pipeline toggles are idempotent; audio only on the primary display; mic start/stop
  c.handle({ type: 'pipelineControl', pipeline: 'video', enabled: false });
  assert.equal(h.sent.filter((m) => m === 'STOP_VIDEO').length, 1);
  c.handle({ type: 'pipelineControl', pipeline: 'audio', enabled: true });
  c.handle({ type: 'pipelineControl', pipeline: 'microphone', enabled: true });
  assert.equal(h.sent.includes('START_AUDIO'), false);   // state already on (pipelineStatusUpdate)
  assert.deepEqual(h.calls.filter((x) => x[0] === 'startMic').length, 1);
  const h2 = mkHost({ displayId: 'display2' });
  new ControlApi(h2).handle({ type: 'pipelineControl', pipeline: 'audio', enabled: true });
  assert.deepEqual(h2.sent, []);
  // shared (view-only) clients ignore everything that would drive the session
  const hs = mkHost({ shared: true });
  const cs = new ControlApi(hs);
  for (const m of [{ type: 'command', value: 'rm' }, { type: 'setManualResolution', width: 800, height: 600 },
    { type: 'pipelineControl', pipeline: 'video', enabled: false }, { type: 'clipboardUpdateFromUI', text: 'x' },
    { type: 'settings', settings: { encoder: 'jpeg' } }]) assert.equal(cs.handle(m), true);
  assert.deepEqual(hs.sent, []);
  assert.equal(hs.calls.length, 0);

  // decoder fallback: 3 errors within 10 s -> reset + reload once
  const fb = new FallbackPolicy();
  assert.equal(fb.onError(0, false), null);
  assert.equal(fb.onError(20000, false), null);   // the first one aged out
  assert.equal(fb.onError(21000, false), null);
  assert.deepEqual(fb.onError(22000, false), { resetSettings: true, reloadAfterMs: 3000 });
  assert.equal(fb.onError(22001, false), null);
  assert.equal(new FallbackPolicy(1).onError(0, true).resetSettings, false);
  assert.equal(SAFE_DEFAULTS.encoder, 'x264enc');

  // shared-mode probing
  const pr = new SharedProbe(1000, 3);
  pr.reset(0);
  assert.deepEqual(pr.tick(500), []);
  assert.deepEqual(pr.tick(1000), ['STOP_VIDEO', 'START_VIDEO']);
  assert.deepEqual(pr.tick(2000), ['STOP_VIDEO', 'START_VIDEO']);
  assert.deepEqual(pr.tick(3000), []);
  assert.equal(pr.state, 'error');
  const pr2 = new SharedProbe(1000, 3);
  pr2.reset(0);
  pr2.onVideo();
  assert.deepEqual(pr2.tick(5000), []);
  assert.equal(pr2.state, 'streaming');

  // IME: nothing during composition, the committed text as keysyms at the end
  const out = [];
  const ime = new ImeComposer((m) => out.push(m));
  ime.start();
  assert.equal(ime.end('日本'), 2);
  assert.deepEqual(out, ['kd,16803301', 'ku,16803301', 'kd,16803628', 'ku,16803628']);
}
console.log('client tests ok');

// ---- WebRTC mode (lib/webrtc.js) with fake WebSocket / RTCPeerConnection ----
import { Signalling, WebRTCClient, parseServerMessage, mungeAnswerSdp, summariseStats } from '../../selkies_gstreamer_amd/web/lib/webrtc.js';

class FakeWS {
  constructor(url) { this.url = url; this.sent = []; FakeWS.last = this; }
  send(m) { this.sent.push(m); }
}
class FakeChannel {
  constructor() { this.readyState = 'open'; this.sent = []; }
  send(m) { this.sent.push(m); }
  close() { this.readyState = 'closed'; }
}
class FakePC {
  constructor(cfg) { this.cfg = cfg; this.remote = null; this.candidates = []; FakePC.last = this; }
  async setRemoteDescription(d) { this.remote = d; }
  async createAnswer() { return { type: 'answer', sdp: 'v=0 answer' }; }
  async setLocalDescription(d) { this.localDescription = d; }
  async addIceCandidate(c) { this.candidates.push(c); }
  close() { this.closed = true; }
}

(async () => {
  const sig = new Signalling('ws://h/ws', 1, FakeWS);
  sig.connect({ res: '1x1' });
  FakeWS.last.onopen();
  assert.ok(FakeWS.last.sent[0].startsWith('HELLO 1 '));
  const statuses = [];
  sig.onstatus = (s) => statuses.push(s);
  sig.handle('HELLO');
  sig.handle('SESSION_OK');
  assert.equal(statuses.length, 2);
  let err = null;
  sig.onerror = (e) => { err = e; };
  sig.handle("ERROR peer '1' not found");
  assert.ok(err && err.message.startsWith('ERROR'));

  const client = new WebRTCClient(null, sig, { iceServers: [] }, FakePC);
  await client.onSdp({ type: 'offer', sdp: 'v=0 offer' });
  assert.equal(FakePC.last.remote.sdp, 'v=0 offer');
  assert.deepEqual(JSON.parse(FakeWS.last.sent[FakeWS.last.sent.length - 1]), { sdp: { type: 'answer', sdp: 'v=0 answer' } });
  sig.handle(JSON.stringify({ ice: { candidate: 'candidate:1 1 udp 1 10.0.0.1 9 typ host', sdpMLineIndex: 0 } }));
  await new Promise((r) => setTimeout(r, 0));
  assert.equal(FakePC.last.candidates.length, 1);

  const ch = new FakeChannel();
  client.bindChannel(ch);
  ch.onmessage({ data: JSON.stringify({ type: 'system', data: { action: 'framerate,60' } }) });
  ch.onmessage({ data: JSON.stringify({ type: 'system', data: { action: 'resolution,1920x1080' } }) });
  ch.onmessage({ data: JSON.stringify({ type: 'ping', data: { start_time: 12.5 } }) });
  assert.equal(client.state.framerate, 60);
  assert.equal(client.state.resolution, '1920x1080');
  assert.equal(ch.sent[0], 'pong,12.5');
  client.setVideoBitrate(2500.7);
  client.requestResolution(1921, 1081);
  assert.deepEqual(ch.sent.slice(1), ['vb,2500', 'r,1920x1080']);
  assert.equal(parseServerMessage('nope'), null);
  // answer munging (reference webrtc.js:271-320)
  const ans = 'a=fmtp:102 level-asymmetry-allowed=1;packetization-mode=1;profile-level-id=42e01f\r\n' +
    'a=fmtp:111 minptime=20;useinbandfec=1\r\n';
  const m = mungeAnswerSdp(ans);
  assert.ok(m.includes('sps-pps-idr-in-keyframe=1;packetization-mode=1'));
  assert.ok(m.includes('minptime=10;') && !m.includes('minptime=20'));
  assert.ok(m.includes('stereo=1;useinbandfec=1'));
  assert.equal(mungeAnswerSdp(m), m);   // idempotent
  assert.ok(mungeAnswerSdp('a=fmtp:102 sps-pps-idr-in-keyframe=0;packetization-mode=1\r\n').includes('sps-pps-idr-in-keyframe=1;'));
  const multi = 'a=rtpmap:100 multiopus/48000/6\r\na=fmtp:100 useinbandfec=1\r\n';
  assert.equal(mungeAnswerSdp(multi), multi);
  // the answer the client sends is the munged one
  const client2 = new WebRTCClient(null, sig, {}, class extends FakePC { async createAnswer() { return { type: 'answer', sdp: ans }; } });
  await client2.onSdp({ type: 'offer', sdp: 'v=0 offer' });
  assert.ok(JSON.parse(FakeWS.last.sent[FakeWS.last.sent.length - 1]).sdp.sdp.includes('stereo=1'));
  // stats: video from the video peer, audio from the separate audio peer
  const rep = (entries) => ({ forEach: (f) => entries.forEach(f) });
  const vpc = { getStats: async () => rep([{ id: 'c1', type: 'codec', mimeType: 'video/H264', clockRate: 90000 },
    { id: 'v', type: 'inbound-rtp', kind: 'video', framesPerSecond: 59.6, codecId: 'c1' },
    { id: 'p', type: 'candidate-pair', nominated: true, state: 'succeeded', currentRoundTripTime: 0.004 }]) };
  const apc = { getStats: async () => rep([{ id: 'a', type: 'inbound-rtp', kind: 'audio', packetsLost: 3 }]) };
  assert.equal(summariseStats(await vpc.getStats(), 'video').codec.mimeType, 'video/H264');
  const vc = new WebRTCClient(null, sig, {}, FakePC);
  vc.pc = vpc;
  const chv = new FakeChannel();
  vc.channel = chv;
  const st = await vc.reportStats({ pc: apc });
  assert.equal(st.audio.packetsLost, 3);
  assert.equal(st.video.transport.currentRoundTripTime, 0.004);
  assert.equal(chv.sent[0], '_f,60');
  assert.ok(chv.sent[1].startsWith('_stats_video,') && chv.sent[2].startsWith('_stats_audio,'));
  assert.deepEqual(parseServerMessage('{"type":"system","data":{"action":"reload"}}').action, ['reload', '']);
})().then(() => console.log('webrtc client ok'), (e) => { console.error(e); process.exit(1); });

// ---- input library state machines (lib/input.js)
import('../../selkies_gstreamer_amd/web/lib/input.js').then(({ KeyboardTracker, WheelAccumulator, TrackpadGestures, KS }) => {
  const DOWN = 8, UP = 16, RIGHT = 128;   // protocol.js MASK_WHEEL_*
  const sent = [];
  let menu = 0, full = 0;
  const kb = new KeyboardTracker((m) => sent.push(m), {
    onMenuHotkey: () => { menu++; }, onFullscreenHotkey: () => { full++; },
  });
  const ev = (code, key, extra = {}) => Object.assign({ code, key, timeStamp: 0 }, extra);
  // plain key + autorepeat + release
  assert.ok(kb.keydown(ev('KeyA', 'a')));
  assert.ok(kb.keydown(ev('KeyA', 'a', { repeat: true })));
  assert.ok(kb.keyup(ev('KeyA', 'a')));
  assert.deepEqual(sent.splice(0), ['kd,97', 'kd,97', 'ku,97']);
  // AltGr on Windows: ControlLeft + AltRight with one timestamp -> ISO_Level3_Shift, no Ctrl
  kb.keydown(ev('ControlLeft', 'Control', { timeStamp: 100 }));
  kb.keydown(ev('AltRight', 'AltGraph', { timeStamp: 100 }));
  kb.keydown(ev('KeyE', '€', { timeStamp: 101 }));
  kb.keyup(ev('KeyE', '€'));
  kb.keyup(ev('AltRight', 'AltGraph'));
  assert.deepEqual(sent.splice(0), [`kd,${KS.AltGr}`, 'kd,16785580', 'ku,16785580', `ku,${KS.AltGr}`]);
  // a real Ctrl is held back until the next key and then sent first
  kb.keydown(ev('ControlLeft', 'Control', { timeStamp: 200 }));
  kb.keydown(ev('KeyC', 'c', { timeStamp: 260, ctrlKey: true }));
  kb.keyup(ev('KeyC', 'c'));
  kb.keyup(ev('ControlLeft', 'Control'));
  assert.deepEqual(sent.splice(0), [`kd,${KS.CtrlL}`, 'kd,99', 'ku,99', `ku,${KS.CtrlL}`]);
  // a lone Ctrl tap still reaches the server
  kb.keydown(ev('ControlLeft', 'Control', { timeStamp: 300 }));
  kb.keyup(ev('ControlLeft', 'Control'));
  assert.deepEqual(sent.splice(0), [`kd,${KS.CtrlL}`, `ku,${KS.CtrlL}`]);
  // hotkeys are consumed locally
  assert.ok(kb.keydown(ev('KeyM', 'M', { ctrlKey: true, shiftKey: true })));
  assert.ok(kb.keydown(ev('KeyF', 'F', { ctrlKey: true, shiftKey: true })));
  assert.deepEqual([menu, full, sent.length], [1, 1, 0]);
  // composition keydowns are ignored; unidentified keys pulse
  assert.equal(kb.keydown(ev('KeyA', 'Process', { keyCode: 229 })), false);
  kb.keydown(ev('Unidentified', 'x'));
  assert.deepEqual(sent.splice(0), ['kd,120', 'ku,120']);
  // macOS: Cmd maps to Ctrl, releasing Cmd releases keys pressed under it
  const mac = new KeyboardTracker((m) => sent.push(m), { macCmdSwap: true });
  mac.keydown(ev('MetaLeft', 'Meta'));
  mac.keydown(ev('KeyV', 'v', { metaKey: true }));
  mac.keyup(ev('MetaLeft', 'Meta'));
  assert.deepEqual(sent.splice(0), [`kd,${KS.CtrlL}`, 'kd,118', `ku,${KS.CtrlL}`, 'ku,118']);
  // blur: everything released, then the server-side reset
  kb.keydown(ev('ShiftLeft', 'Shift'));
  kb.keydown(ev('KeyQ', 'Q', { shiftKey: true }));
  kb.reset();
  assert.deepEqual(sent.splice(0), ['kd,65505', 'kd,81', 'ku,65505', 'ku,81', 'kr']);
  // typed text / mobile virtual keyboard
  kb.typeText('Hi');
  assert.deepEqual(sent.splice(0), ['kd,65505', 'kd,72', 'ku,72', 'ku,65505', 'kd,105', 'ku,105']);
  kb.mobileInput({ inputType: 'deleteContentBackward' });
  kb.mobileInput({ inputType: 'insertText', data: 'é' });
  assert.deepEqual(sent.splice(0), ['kd,65288', 'ku,65288', 'kd,233', 'ku,233']);

  // wheel: line-mode notches and accumulated fine trackpad deltas
  const w = new WheelAccumulator();
  assert.deepEqual(w.feed({ deltaY: 3, deltaMode: 1 }), [{ bit: DOWN, magnitude: 1 }]);   // 120 px -> 1 notch, 20 left
  assert.deepEqual(w.feed({ deltaY: 30, deltaMode: 0 }), []);
  assert.deepEqual(w.feed({ deltaY: 60, deltaMode: 0 }), [{ bit: DOWN, magnitude: 1 }]);
  assert.deepEqual(w.feed({ deltaY: -250, deltaMode: 0 }), [{ bit: UP, magnitude: 2 }]);  // direction change resets
  assert.deepEqual(w.feed({ deltaX: 100, deltaMode: 0 }).map((p) => p.bit), [RIGHT]);

  // trackpad gestures
  const g = new TrackpadGestures();
  const T = (id, x, y) => ({ identifier: id, clientX: x, clientY: y });
  assert.deepEqual(g.handle('touchstart', [T(1, 10, 10)], 0), []);
  assert.deepEqual(g.handle('touchend', [T(1, 10, 10)], 100), [{ button: 1, down: true }, { button: 1, down: false }]);
  // touch again right after a tap: drag with the button held
  assert.deepEqual(g.handle('touchstart', [T(2, 10, 10)], 200), [{ button: 1, down: true }]);
  assert.deepEqual(g.handle('touchmove', [T(2, 40, 10)], 250), [{ move: [45, 0] }]);
  assert.deepEqual(g.handle('touchend', [T(2, 40, 10)], 600), [{ button: 1, down: false }]);
  // one-finger move below the tap slop does nothing; beyond it moves relatively
  g.handle('touchstart', [T(3, 0, 0)], 2000);
  assert.deepEqual(g.handle('touchmove', [T(3, 4, 0)], 2010), []);
  assert.deepEqual(g.handle('touchmove', [T(3, 20, 0)], 2020), [{ move: [24, 0] }]);
  assert.deepEqual(g.handle('touchend', [T(3, 20, 0)], 2030), []);
  // two-finger tap = right click, two-finger drag = scroll, three-finger tap = middle click
  g.handle('touchstart', [T(4, 0, 100), T(5, 50, 100)], 3000);
  assert.deepEqual(g.handle('touchend', [T(4, 0, 100), T(5, 50, 100)], 3050), [{ button: 4, down: true }, { button: 4, down: false }]);
  g.handle('touchstart', [T(6, 0, 100), T(7, 50, 100)], 4000);
  const sc = g.handle('touchmove', [T(6, 0, 40), T(7, 50, 40)], 4050);
  assert.equal(sc.length, 2);
  assert.deepEqual(sc[0], { wheel: DOWN, magnitude: 1 });   // fingers up: content scrolls down
  g.handle('touchend', [T(6, 0, 40), T(7, 50, 40)], 4100);
  g.handle('touchstart', [T(8, 0, 0), T(9, 20, 0), T(10, 40, 0)], 5000);
  assert.deepEqual(g.handle('touchend', [T(8, 0, 0), T(9, 20, 0), T(10, 40, 0)], 5050), [{ button: 2, down: true }, { button: 2, down: false }]);
  console.log('input lib ok');
}).catch((e) => { console.error(e); process.exit(1); });

// ---- dashboard layouts, gamepad visualiser, system monitor
assert.equal(dash.pickLayout('', {}), 'selkies');
assert.equal(dash.pickLayout('?x=1&ui=wish', { ui_dashboard: { value: 'zinc' } }), 'wish');
assert.equal(dash.pickLayout('', { ui_dashboard: { value: 'zinc' } }), 'zinc');
assert.equal(dash.pickLayout('?ui=bogus', { ui_dashboard: 'nope' }), 'selkies');
assert.deepEqual(Object.keys(dash.LAYOUTS), ['selkies', 'zinc', 'wish']);
{
  const pad = { buttons: [{ pressed: true, value: 1 }, { pressed: false, value: 0 }], axes: [1, -1, 0, 0.5] };
  const sh = dash.padShapes(pad);
  assert.equal(sh.filter((x) => x.kind === 'button').length, 17);
  assert.equal(sh[0].on, true);
  assert.equal(sh[1].on, false);
  const sticks = sh.filter((x) => x.kind === 'stick');
  assert.deepEqual([sticks[0].x, sticks[0].y, sticks[1].x, sticks[1].y], [80, 76, 128, 88]);
  const svg = dash.padSvg(pad);
  assert.ok(svg.startsWith('<svg') && (svg.match(/<circle/g) || []).length === 19);
  const g = dash.monitorGauges({ cpu: 50, mem: 0.25, gpu: 1.7, vram: null });
  assert.deepEqual(g.map((x) => x.value), [0.5, 0.25, 1, null]);
}
console.log('dashboard layouts ok');

// ---- i18n (reference translations.js languages) and the apps panel helpers
import('../../selkies_gstreamer_amd/web/lib/i18n.js').then((i18n) => {
  const langs = Object.keys(i18n.LANGUAGES);
  assert.deepEqual(langs, ['en', 'es', 'zh', 'hi', 'pt', 'fr', 'ru', 'de', 'tr', 'it', 'nl', 'ar', 'ko', 'ja', 'vi', 'th',
    'fil', 'da']);
  const keys = Object.keys(i18n.LANGUAGES.en);
  for (const l of langs) {
    assert.deepEqual(Object.keys(i18n.LANGUAGES[l]).sort(), keys.slice().sort(), `keys of ${l}`);
    assert.ok(i18n.LANGUAGE_NAMES[l], `name of ${l}`);
    for (const k of keys) if (k.endsWith('player')) assert.ok(i18n.LANGUAGES[l][k].includes('{n}'), `${l} ${k}`);
  }
  assert.equal(i18n.pickLanguage('?lang=ja', ['fr']), 'ja');
  assert.equal(i18n.pickLanguage('', ['xx-YY', 'pt-BR', 'de']), 'pt');
  assert.equal(i18n.pickLanguage('?lang=zz', []), 'en');
  const de = i18n.translator('de-DE');
  assert.equal(de.lang, 'de');
  assert.equal(de('sharing.player', { n: 3 }), 'Spieler 3');
  assert.equal(de('no.such.key'), 'no.such.key');
  assert.equal(i18n.translator('xx')('section.files'), 'Files');
  assert.equal(i18n.isRtl('ar'), true);
  assert.equal(i18n.isRtl('fr'), false);
  const links = dash.sharingLinks('http://h/p#x', { enable_sharing: true, enable_shared: true, enable_player2: true,
    enable_player3: false, enable_player4: false }, i18n.translator('fr'));
  assert.deepEqual(links.map((x) => x.label), ['lecture seule', 'joueur 2']);
  console.log('i18n ok');
  return import('../../selkies_gstreamer_amd/web/lib/apps.js');
}).then((apps) => {
  const cat = apps.parseCatalog({ apps: [
    { name: 'firefox', full_name: 'Firefox', description: 'Web browser', icon: 'ff.png' },
    { name: 'gimp', description: 'Image editor' },
    { name: 'evil; rm -rf /', full_name: 'bad' },
    { full_name: 'no name' },
  ] });
  assert.deepEqual(cat.map((a) => a.name), ['firefox', 'gimp']);
  assert.equal(cat[1].title, 'gimp');
  assert.deepEqual(apps.filterApps(cat, 'BROWSER').map((a) => a.name), ['firefox']);
  assert.deepEqual(apps.filterApps(cat, '').map((a) => a.name), ['firefox', 'gimp']);
  assert.equal(apps.appCommand('install', 'firefox'), 'cmd,st ~/.local/bin/proot-apps install firefox');
  assert.throws(() => apps.appCommand('install', 'a b'));
  assert.throws(() => apps.appCommand('format', 'firefox'));
  const store = { v: {}, getItem(k) { return this.v[k] || null; }, setItem(k, x) { this.v[k] = x; } };
  let inst = apps.loadInstalled(store);
  assert.deepEqual(inst, []);
  inst = apps.updateInstalled(inst, 'install', 'gimp');
  inst = apps.updateInstalled(inst, 'install', 'firefox');
  inst = apps.updateInstalled(inst, 'install', 'gimp');
  apps.saveInstalled(store, inst);
  assert.deepEqual(apps.loadInstalled(store), ['firefox', 'gimp']);
  assert.deepEqual(apps.updateInstalled(inst, 'remove', 'gimp'), ['firefox']);
  store.v[apps.INSTALLED_KEY] = '{bad json';
  assert.deepEqual(apps.loadInstalled(store), []);
  console.log('apps ok');
});

// ---- codec strings of the negotiated encoder (lib/video.js)
import('../../selkies_gstreamer_amd/web/lib/video.js').then(({ codecString }) => {
  assert.equal(codecString('x264enc', 1920, 1080, 60), 'avc1.42E01E');
  assert.equal(codecString('x264enc-striped', 1920, 64, 60), 'avc1.42E01E');
  assert.equal(codecString('x265enc', 1920, 1080, 60), 'hev1.1.6.L123.B0');   // 1920x1088 coded: level 4.1
  assert.equal(codecString('x265enc', 3840, 2160, 60), 'hev1.1.6.L153.B0');   // level 5.1
  assert.equal(codecString('svtav1enc', 3840, 2160, 120), 'av01.0.14M.08');   // level 5.2
  assert.equal(codecString('svtav1enc', 1920, 1080, 60), 'av01.0.09M.08');    // level 4.1 (4.0 tops out at 30 fps)
  console.log('codec strings ok');
}).catch((e) => { console.error(e); process.exit(1); });

// ---- decode-queue drop: no delta after a drop is decoded before the next key frame, and a
// key frame is requested (lib/video.js VideoRenderer.h264)
import('../../selkies_gstreamer_amd/web/lib/video.js').then(({ VideoRenderer, KEY_REQUEST_INTERVAL_MS }) => {
  if (typeof globalThis.performance === 'undefined') globalThis.performance = { now: () => Date.now() };
  const decoded = [];
  let queue = 0;
  globalThis.EncodedVideoChunk = class { constructor(o) { Object.assign(this, o); } };
  globalThis.VideoDecoder = class {
    constructor() { this.state = 'configured'; }
    configure() {}
    get decodeQueueSize() { return queue; }
    decode(c) { decoded.push(c.data[0]); }
    close() { this.state = 'closed'; }
  };
  const canvas = { width: 0, height: 0, getContext: () => ({ fillRect() {}, drawImage() {} }) };
  const requests = [];
  const v = new VideoRenderer(canvas, null, (y) => requests.push(y));
  const pkt = (n, key) => ({ frameId: n, y: 0, width: 1920, height: 1080, key, payload: new Uint8Array([n]) });
  v.h264(pkt(0, true));
  // 40 queued deltas: the decoder falls behind at delta 10 and recovers at delta 20
  for (let n = 1; n <= 40; n++) {
    queue = n >= 10 && n < 20 ? 31 : 0;
    v.h264(pkt(n, false));
  }
  assert.deepEqual(decoded, [0, ...Array.from({ length: 9 }, (_, i) => i + 1)]);   // nothing after the drop
  assert.ok(requests.length >= 1 && requests.every((y) => y === 0));
  assert.ok(requests.length <= 2);   // rate limited (KEY_REQUEST_INTERVAL_MS)
  assert.ok(KEY_REQUEST_INTERVAL_MS > 0 && v.dropped === 1);   // the rest wait unkeyed
  v.h264(pkt(41, true));             // the requested key frame resumes decoding
  v.h264(pkt(42, false));
  assert.deepEqual(decoded.slice(-2), [41, 42]);
  console.log('decode-drop resync ok');
}).catch((e) => { console.error(e); process.exit(1); });

