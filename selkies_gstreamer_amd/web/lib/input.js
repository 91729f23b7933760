// Keyboard, pointer, pen, wheel, touch/trackpad, virtual-keyboard and gamepad
// capture -> server input messages (vocabulary handled by server/input.py:
// kd/ku/kr, m/m2, js,c|d|b|a).
//
// Behaviour parity with the reference client input library
// (addons/gst-web-core/lib/input.js): keydown/keyup bookkeeping with stuck-key
// release (1300-1496), the Windows AltGr = ControlLeft+AltRight pair (1359-1366,
// 1475-1480), macOS Cmd handling (1378-1390, 1466-1472), Ctrl+Shift+M / F hotkeys
// (1341-1356), IME composition and mobile virtual-keyboard text (1498-1571), pen
// pointer events (1663-1683), trackpad gestures (1685-1800) and wheel
// normalisation. The gesture and keyboard state machines are plain classes with
// no DOM dependency so they are unit tested under node (tests/js/client_test.mjs).
import { charToKeysym, keysymFor } from './keysyms.js';
import {
  MASK_WHEEL_DOWN, MASK_WHEEL_LEFT, MASK_WHEEL_RIGHT, MASK_WHEEL_UP, buttonBit, mouseMessage, toStreamCoords, utf8ToB64,
} from './protocol.js';

const GAMEPAD_POLL_MS = 16;
const WHEEL_MAX_MAGNITUDE = 10;
const WHEEL_LINE_PX = 40;        // DOM_DELTA_LINE -> pixels
const WHEEL_PAGE_PX = 800;       // DOM_DELTA_PAGE -> pixels
const WHEEL_STEP_PX = 100;       // one notch of a classic wheel

export const KS = {
  ShiftL: 0xffe1, ShiftR: 0xffe2, CtrlL: 0xffe3, CtrlR: 0xffe4, AltL: 0xffe9, AltR: 0xffea,
  MetaL: 0xffeb, MetaR: 0xffec, SuperL: 0xffeb, AltGr: 0xfe03, BackSpace: 0xff08, Return: 0xff0d,
};

// ---------------------------------------------------------------------------
// Keyboard state machine
// ---------------------------------------------------------------------------
// keydown(ev) / keyup(ev) take KeyboardEvent-like objects ({key, code, repeat,
// ctrlKey, shiftKey, timeStamp, isComposing, keyCode}) and return true when the
// event was consumed (the caller then calls preventDefault).
export class KeyboardTracker {
  constructor(send, opts = {}) {
    this.send = send;
    this.down = new Map();             // code -> keysym sent on keydown
    this.macCmdSwap = !!opts.macCmdSwap; // Cmd acts as Ctrl for the remote (macOS clients)
    this.onMenuHotkey = opts.onMenuHotkey || null;
    this.onFullscreenHotkey = opts.onFullscreenHotkey || null;
    this.composing = false;
    this._altGr = null;                // pending ControlLeft {ts}: maybe the first half of AltGr
  }

  _press(code, ks) {
    this.down.set(code, ks);
    this.send(`kd,${ks}`);
  }

  _release(code) {
    const ks = this.down.get(code);
    if (ks === undefined) return false;
    this.down.delete(code);
    this.send(`ku,${ks}`);
    return true;
  }

  _keysym(ev) {
    const code = ev.code || '';
    if (this.macCmdSwap && (code === 'MetaLeft' || code === 'OSLeft')) return KS.CtrlL;
    if (this.macCmdSwap && (code === 'MetaRight' || code === 'OSRight')) return KS.CtrlR;
    return keysymFor(ev);
  }

  // A pending ControlLeft that did not turn out to be AltGr is a real Ctrl press.
  _flushAltGr() {
    if (this._altGr) {
      this._altGr = null;
      this._press('ControlLeft', KS.CtrlL);
    }
  }

  keydown(ev) {
    if (ev.isComposing || ev.keyCode === 229 || this.composing) return false;
    const code = ev.code || ev.key || '';
    if (ev.ctrlKey && ev.shiftKey && !ev.repeat) {
      if (code === 'KeyM' && this.onMenuHotkey) { this.onMenuHotkey(); return true; }
      if (code === 'KeyF' && this.onFullscreenHotkey) { this.onFullscreenHotkey(); return true; }
    }
    // Windows reports AltGr as ControlLeft immediately followed by AltRight
    // with the same timestamp: hold the Ctrl back until the next key decides.
    if (code === 'ControlLeft' && !ev.repeat && !this.down.has(code)) {
      this._flushAltGr();
      this._altGr = { ts: ev.timeStamp };
      return true;
    }
    if (this._altGr) {
      const pending = this._altGr;
      if (code === 'AltRight' && ev.timeStamp !== undefined && Math.abs(ev.timeStamp - pending.ts) < 2) {
        this._altGr = null;
        this._press('AltRight', KS.AltGr);
        return true;
      }
      this._flushAltGr();
    }
    const ks = this._keysym(ev);
    if (ks === null || ks === undefined) return false;
    if (code === 'Unidentified' || !ev.code) {
      // No matching keyup will identify this key (virtual keyboards): pulse it.
      this.send(`kd,${ks}`);
      this.send(`ku,${ks}`);
      return true;
    }
    const prev = this.down.get(code);
    if (prev !== undefined && prev !== ks) this._release(code);   // layout/modifier change mid-hold
    if (ev.repeat && prev === ks) {
      this.send(`kd,${ks}`);         // autorepeat
      return true;
    }
    this._press(code, ks);
    return true;
  }

  keyup(ev) {
    const code = ev.code || ev.key || '';
    if (code === 'ControlLeft' && this._altGr) this._flushAltGr();
    else if (this._altGr) this._flushAltGr();
    let handled = this._release(code);
    if (!handled) {
      const ks = this._keysym(ev);
      if (ks !== null && ks !== undefined && code !== 'Unidentified') {
        this.send(`ku,${ks}`);
        handled = true;
      }
    }
    // macOS delivers no keyup for keys released while Cmd is held: releasing
    // Cmd releases everything that was pressed with it.
    if (code === 'MetaLeft' || code === 'MetaRight' || code === 'OSLeft' || code === 'OSRight') {
      for (const c of [...this.down.keys()]) {
        if (!/^(Shift|Control|Alt)/.test(c)) this._release(c);
      }
    }
    return handled;
  }

  // Window blur / visibility loss: nothing may stay pressed on the remote.
  reset() {
    this._altGr = null;
    for (const c of [...this.down.keys()]) this._release(c);
    this.send('kr');
  }

  // Typed text (IME commit, mobile virtual keyboards, paste-as-keystrokes):
  // one down/up pulse per character; ASCII capitals are typed with Shift held.
  typeText(text) {
    for (const ch of text) {
      if (ch === '\n') { this.send(`kd,${KS.Return}`); this.send(`ku,${KS.Return}`); continue; }
      const ks = charToKeysym(ch);
      if (ks === null) continue;
      const upper = ch >= 'A' && ch <= 'Z';
      if (upper) this.send(`kd,${KS.ShiftL}`);
      this.send(`kd,${ks}`);
      this.send(`ku,${ks}`);
      if (upper) this.send(`ku,${KS.ShiftL}`);
    }
  }

  backspace(n = 1) {
    for (let i = 0; i < n; i++) { this.send(`kd,${KS.BackSpace}`); this.send(`ku,${KS.BackSpace}`); }
  }

  // `input` events of a hidden text field that a mobile virtual keyboard types into.
  mobileInput(ev) {
    if (ev.inputType === 'deleteContentBackward') { this.backspace(1); return true; }
    if (ev.inputType === 'insertLineBreak') { this.typeText('\n'); return true; }
    if (ev.data) { this.typeText(ev.data); return true; }
    return false;
  }
}

// ---------------------------------------------------------------------------
// Wheel normalisation
// ---------------------------------------------------------------------------
// Turns WheelEvents (pixel, line or page deltas; coarse mouse notches or fine
// trackpad deltas) into wheel pulses {bit, magnitude}. Fine deltas accumulate
// until they make a notch so a trackpad scrolls at the same speed as a wheel.
export class WheelAccumulator {
  constructor() { this.accX = 0; this.accY = 0; }

  static px(delta, mode) {
    if (mode === 1) return delta * WHEEL_LINE_PX;
    if (mode === 2) return delta * WHEEL_PAGE_PX;
    return delta;
  }

  feed(ev) {
    const out = [];
    const dy = WheelAccumulator.px(ev.deltaY || 0, ev.deltaMode || 0);
    const dx = WheelAccumulator.px(ev.deltaX || 0, ev.deltaMode || 0);
    if (Math.sign(dy) !== Math.sign(this.accY)) this.accY = 0;
    if (Math.sign(dx) !== Math.sign(this.accX)) this.accX = 0;
    this.accY += dy;
    this.accX += dx;
    const emit = (acc, neg, pos) => {
      const notches = Math.trunc(Math.abs(acc) / WHEEL_STEP_PX);
      if (!notches) return acc;
      out.push({ bit: acc < 0 ? neg : pos, magnitude: Math.min(WHEEL_MAX_MAGNITUDE, notches) });
      return acc - Math.sign(acc) * notches * WHEEL_STEP_PX;
    };
    this.accY = emit(this.accY, MASK_WHEEL_UP, MASK_WHEEL_DOWN);
    this.accX = emit(this.accX, MASK_WHEEL_LEFT, MASK_WHEEL_RIGHT);
    return out;
  }
}

// ---------------------------------------------------------------------------
// Trackpad gestures (touch screen used like a laptop trackpad)
// ---------------------------------------------------------------------------
// handle(type, touches, changed, now) with touches = [{identifier, clientX,
// clientY}] returns a list of actions:
//   {move: [dx, dy]}            relative pointer motion
//   {button: bit, down: bool}    press / release
//   {wheel: bit, magnitude}      scroll pulse
// One finger moves; a short tap clicks; tap then touch-and-move drags; two
// fingers scroll (tap = right click); three fingers tap = middle click.
export class TrackpadGestures {
  constructor(opts = {}) {
    this.sensitivity = opts.sensitivity || 1.5;
    this.tapMs = opts.tapMs || 220;
    this.tapSlopSq = (opts.tapSlop || 10) ** 2;
    this.scrollStep = opts.scrollStep || 24;
    this.touches = new Map();   // id -> {x, y, x0, y0}
    this.maxFingers = 0;
    this.t0 = 0;
    this.moved = false;
    this.lastTapEnd = -1e9;
    this.dragging = false;
    this.scrollAcc = 0;
    this.lastCentroid = null;
  }

  _centroid() {
    let x = 0, y = 0;
    for (const t of this.touches.values()) { x += t.x; y += t.y; }
    const n = this.touches.size || 1;
    return [x / n, y / n];
  }

  handle(type, changed, now) {
    const out = [];
    if (type === 'touchstart') {
      if (this.touches.size === 0) {
        this.t0 = now;
        this.moved = false;
        this.maxFingers = 0;
        // touch shortly after a tap: this touch drags with the left button held
        if (now - this.lastTapEnd < this.tapMs * 1.5 && changed.length === 1) {
          this.dragging = true;
          out.push({ button: 1, down: true });
        }
      }
      for (const t of changed) {
        this.touches.set(t.identifier, { x: t.clientX, y: t.clientY, x0: t.clientX, y0: t.clientY });
      }
      this.maxFingers = Math.max(this.maxFingers, this.touches.size);
      this.lastCentroid = this.touches.size >= 2 ? this._centroid() : null;
      this.scrollAcc = 0;
    } else if (type === 'touchmove') {
      let dx = 0, dy = 0;
      for (const t of changed) {
        const s = this.touches.get(t.identifier);
        if (!s) continue;
        if ((t.clientX - s.x0) ** 2 + (t.clientY - s.y0) ** 2 > this.tapSlopSq) this.moved = true;
        dx += t.clientX - s.x;
        dy += t.clientY - s.y;
        s.x = t.clientX;
        s.y = t.clientY;
      }
      if (this.touches.size === 1) {
        if (this.moved && (dx || dy)) out.push({ move: [dx * this.sensitivity, dy * this.sensitivity] });
      } else if (this.touches.size === 2 && this.lastCentroid) {
        const c = this._centroid();
        this.scrollAcc += c[1] - this.lastCentroid[1];
        this.lastCentroid = c;
        while (Math.abs(this.scrollAcc) >= this.scrollStep) {
          // natural scrolling: fingers moving up scroll the content down
          out.push({ wheel: this.scrollAcc < 0 ? MASK_WHEEL_DOWN : MASK_WHEEL_UP, magnitude: 1 });
          this.scrollAcc -= Math.sign(this.scrollAcc) * this.scrollStep;
        }
      }
    } else if (type === 'touchend' || type === 'touchcancel') {
      for (const t of changed) this.touches.delete(t.identifier);
      if (this.touches.size === 0) {
        const quick = now - this.t0 < this.tapMs && !this.moved && type === 'touchend';
        if (this.dragging) {
          out.push({ button: 1, down: false });
          this.dragging = false;
          if (quick) {            // double tap: second click
            out.push({ button: 1, down: true }, { button: 1, down: false });
          }
          this.lastTapEnd = -1e9;
        } else if (quick) {
          const bit = this.maxFingers >= 3 ? 2 : this.maxFingers === 2 ? 4 : 1;
          out.push({ button: bit, down: true }, { button: bit, down: false });
          this.lastTapEnd = bit === 1 ? now : -1e9;
        } else {
          this.lastTapEnd = -1e9;
        }
      } else {
        this.lastCentroid = this.touches.size >= 2 ? this._centroid() : null;
      }
    }
    return out;
  }
}

// ---------------------------------------------------------------------------
// DOM binding
// ---------------------------------------------------------------------------
export class Input {
  constructor(element, send, getStreamSize) {
    this.el = element;
    this.send = send;
    this.streamSize = getStreamSize;
    this.mask = 0;
    this.listeners = [];
    this.pads = new Map();      // index -> {buttons:[], axes:[]}
    this.padTimer = null;
    this.enabled = false;
    this.padOffset = 0;         // #player2..4 links map local pads to server slots 1..3
    this.gamepadOnly = false;   // player links: no keyboard / mouse
    this.trackpad = false;      // touch drives a relative pointer like a laptop trackpad
    this.onMenuHotkey = null;
    this.onFullscreenHotkey = null;
    const isMac = typeof navigator !== 'undefined' && /Mac|iPhone|iPad/.test(navigator.platform || '');
    this.keyboard = new KeyboardTracker(send, {
      macCmdSwap: isMac,
      onMenuHotkey: () => this.onMenuHotkey && this.onMenuHotkey(),
      onFullscreenHotkey: () => this.onFullscreenHotkey && this.onFullscreenHotkey(),
    });
    this.wheel = new WheelAccumulator();
    this.gestures = new TrackpadGestures();
    this._lastTouchY = null;
    this._mobileField = null;
  }

  // back-compat: the pressed-key map
  get pressed() { return this.keyboard.down; }

  _on(target, type, fn, opts) {
    const h = fn.bind(this);
    target.addEventListener(type, h, opts);
    this.listeners.push([target, type, h, opts]);
  }

  attach() {
    if (this.enabled) return;
    this.enabled = true;
    this._on(window, 'gamepadconnected', this._padConnected);
    this._on(window, 'gamepaddisconnected', this._padDisconnected);
    this.padTimer = setInterval(() => this._pollPads(), GAMEPAD_POLL_MS);
    if (this.gamepadOnly) return;
    this._on(window, 'keydown', this._keydown, true);
    this._on(window, 'keyup', this._keyup, true);
    this._on(window, 'blur', this.releaseAll);
    this._on(document, 'visibilitychange', () => { if (document.hidden) this.releaseAll(); });
    // composed text itself is typed by the client's ImeComposer (control.js)
    this._on(window, 'compositionstart', () => { this.keyboard.composing = true; }, true);
    this._on(window, 'compositionend', () => { this.keyboard.composing = false; }, true);
    this._on(this.el, 'mousemove', this._mousemove);
    this._on(this.el, 'mousedown', this._mousebutton);
    this._on(this.el, 'mouseup', this._mousebutton);
    this._on(this.el, 'pointerdown', this._pen);
    this._on(this.el, 'pointermove', this._pen);
    this._on(this.el, 'pointerup', this._pen);
    this._on(this.el, 'wheel', this._wheel, { passive: false });
    this._on(this.el, 'contextmenu', (e) => e.preventDefault());
    this._on(this.el, 'touchstart', this._touch, { passive: false });
    this._on(this.el, 'touchmove', this._touch, { passive: false });
    this._on(this.el, 'touchend', this._touch, { passive: false });
    this._on(this.el, 'touchcancel', this._touch, { passive: false });
  }

  detach() {
    for (const [t, type, h, opts] of this.listeners) t.removeEventListener(type, h, opts);
    this.listeners = [];
    clearInterval(this.padTimer);
    this.enabled = false;
  }

  releaseAll() {
    this.keyboard.reset();
    if (this.mask & 7) {
      this.mask = 0;
      this.send(mouseMessage(true, 0, 0, 0));
    }
  }

  // ---------------------------------------------------------------- keyboard
  _keydown(e) {
    if (this.keyboard.keydown(e)) e.preventDefault();
  }

  _keyup(e) {
    if (this.keyboard.keyup(e)) e.preventDefault();
  }

  typeText(text) { this.send(`co,end,${text}`); }

  // Shows the virtual keyboard on touch devices through a hidden text field and
  // forwards what is typed into it.
  showVirtualKeyboard() {
    if (!this._mobileField) {
      const f = document.createElement('textarea');
      f.setAttribute('autocapitalize', 'off');
      f.setAttribute('autocomplete', 'off');
      f.style.cssText = 'position:fixed;left:-1000px;top:0;opacity:0;width:1px;height:1px';
      document.body.appendChild(f);
      f.addEventListener('input', (e) => { this.keyboard.mobileInput(e); f.value = ''; });
      this._mobileField = f;
    }
    this._mobileField.focus();
  }

  // ---------------------------------------------------------------- pointer
  _pos(e) {
    const r = this.el.getBoundingClientRect();
    const [sw, sh] = this.streamSize();
    return toStreamCoords(e.clientX - r.left, e.clientY - r.top, r.width, r.height, sw, sh);
  }

  _locked() { return typeof document !== 'undefined' && document.pointerLockElement === this.el; }

  _mousemove(e) {
    if (this._locked()) {
      this.send(mouseMessage(true, e.movementX, e.movementY, this.mask));
    } else {
      // the most recent of the coalesced moves is the one that matters
      const evs = e.getCoalescedEvents ? e.getCoalescedEvents() : null;
      const last = evs && evs.length ? evs[evs.length - 1] : e;
      const [x, y] = this._pos(last);
      this.send(mouseMessage(false, x, y, this.mask));
    }
  }

  _mousebutton(e) {
    e.preventDefault();
    // Ctrl+Shift+left click toggles pointer lock (relative mouse for games)
    if (e.type === 'mousedown' && e.button === 0 && e.ctrlKey && e.shiftKey) {
      if (this._locked()) document.exitPointerLock(); else this.requestPointerLock();
      return;
    }
    const bit = buttonBit(e.button);
    if (e.type === 'mousedown') this.mask |= bit; else this.mask &= ~bit;
    if (this._locked()) {
      this.send(mouseMessage(true, 0, 0, this.mask));
    } else {
      const [x, y] = this._pos(e);
      this.send(mouseMessage(false, x, y, this.mask));
    }
  }

  // Pen / stylus: absolute pointer with the tip as the left button (mouse and
  // touch pointers are handled by their own events).
  _pen(e) {
    if (e.pointerType !== 'pen') return;
    e.preventDefault();
    if (e.type === 'pointerdown') this.mask |= buttonBit(e.button < 0 ? 0 : e.button);
    else if (e.type === 'pointerup') this.mask &= ~buttonBit(e.button < 0 ? 0 : e.button);
    const [x, y] = this._pos(e);
    this.send(mouseMessage(false, x, y, this.mask));
  }

  _wheelPulse(bit, magnitude) {
    magnitude = Math.max(1, Math.min(WHEEL_MAX_MAGNITUDE, Math.round(magnitude)));
    this.send(mouseMessage(true, 0, 0, this.mask | bit, magnitude));
    setTimeout(() => this.send(mouseMessage(true, 0, 0, this.mask & ~bit, magnitude)), 10);
  }

  _wheel(e) {
    e.preventDefault();
    for (const p of this.wheel.feed(e)) this._wheelPulse(p.bit, p.magnitude);
  }

  _applyGesture(actions) {
    for (const a of actions) {
      if (a.move) {
        this.send(mouseMessage(true, a.move[0], a.move[1], this.mask));
      } else if (a.button) {
        if (a.down) this.mask |= a.button; else this.mask &= ~a.button;
        this.send(mouseMessage(true, 0, 0, this.mask));
      } else if (a.wheel) {
        this._wheelPulse(a.wheel, a.magnitude);
      }
    }
  }

  // Touch: trackpad gestures, or direct touch (one finger = left-button drag at
  // the finger, two fingers = vertical scroll).
  _touch(e) {
    e.preventDefault();
    if (this.trackpad) {
      this._applyGesture(this.gestures.handle(e.type, [...e.changedTouches], performance.now()));
      return;
    }
    const t = e.touches;
    if (t.length === 1) {
      const [x, y] = this._pos(t[0]);
      const down = e.type !== 'touchend';
      this.mask = down ? (this.mask | 1) : (this.mask & ~1);
      this.send(mouseMessage(false, x, y, this.mask));
      this._lastTouchY = null;
    } else if (t.length === 2) {
      const y = (t[0].clientY + t[1].clientY) / 2;
      if (this._lastTouchY != null && Math.abs(y - this._lastTouchY) > 12) {
        this._wheelPulse(y < this._lastTouchY ? MASK_WHEEL_DOWN : MASK_WHEEL_UP, 1);
        this._lastTouchY = y;
      } else if (this._lastTouchY == null) {
        this._lastTouchY = y;
      }
    } else if ((e.type === 'touchend' || e.type === 'touchcancel') && this.mask & 1) {
      this.mask &= ~1;
      this.send(mouseMessage(true, 0, 0, this.mask));
    }
  }

  requestPointerLock() {
    if (this.el.requestPointerLock) this.el.requestPointerLock();
  }

  // ---------------------------------------------------------------- gamepads
  _padConnected(e) {
    const gp = e.gamepad;
    if (gp.index > 3) return;
    this.pads.set(gp.index, { buttons: gp.buttons.map(() => 0), axes: gp.axes.map(() => 0) });
    this.send(`js,c,${this._slot(gp.index)},${utf8ToB64(gp.id.slice(0, 255))},${gp.axes.length},${gp.buttons.length}`);
  }

  _padDisconnected(e) {
    if (!this.pads.has(e.gamepad.index)) return;
    this.pads.delete(e.gamepad.index);
    this.send(`js,d,${this._slot(e.gamepad.index)}`);
  }

  _slot(index) { return Math.min(3, index + this.padOffset); }

  _pollPads() {
    if (this.gamepadsEnabled === false) return;   // gamepadControl {enabled: false} (control.js)
    if (!navigator.getGamepads || !this.pads.size) return;
    for (const gp of navigator.getGamepads()) {
      if (!gp || !this.pads.has(gp.index)) continue;
      const st = this.pads.get(gp.index);
      gp.buttons.forEach((b, i) => {
        const v = Math.round(b.value * 100) / 100;
        if (v !== st.buttons[i]) {
          st.buttons[i] = v;
          this.send(`js,b,${this._slot(gp.index)},${i},${v}`);
        }
      });
      gp.axes.forEach((a, i) => {
        const v = Math.round(a * 100) / 100;
        if (v !== st.axes[i]) {
          st.axes[i] = v;
          this.send(`js,a,${this._slot(gp.index)},${i},${v}`);
        }
      });
    }
  }
}
