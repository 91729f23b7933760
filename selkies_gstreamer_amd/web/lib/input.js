// Keyboard, pointer, wheel, touch and gamepad capture -> server input messages
// (vocabulary handled by server/input.py: kd/ku/kr, m/m2, js,c|d|b|a).
import { keysymFor } from './keysyms.js';
import {
  MASK_WHEEL_DOWN, MASK_WHEEL_LEFT, MASK_WHEEL_RIGHT, MASK_WHEEL_UP, buttonBit, mouseMessage, toStreamCoords, utf8ToB64,
} from './protocol.js';

const GAMEPAD_POLL_MS = 16;
const WHEEL_MAX_MAGNITUDE = 10;

export class Input {
  constructor(element, send, getStreamSize) {
    this.el = element;
    this.send = send;
    this.streamSize = getStreamSize;
    this.mask = 0;
    this.pressed = new Map();   // code -> keysym (release what was pressed)
    this.listeners = [];
    this.pads = new Map();      // index -> {buttons:[], axes:[]}
    this.padTimer = null;
    this.smallestWheel = 100;
    this.enabled = false;
    this.padOffset = 0;         // #player2..4 links map local pads to server slots 1..3
    this.gamepadOnly = false;   // player links: no keyboard / mouse
    this.trackpad = false;      // touch drives a relative pointer like a laptop trackpad
    this._tp = null;
  }

  _on(target, type, fn, opts) {
    const h = fn.bind(this);
    target.addEventListener(type, h, opts);
    this.listeners.push([target, type, h, opts]);
  }

  attach() {
    if (this.enabled) return;
    this.enabled = true;
    if (this.gamepadOnly) {
      this._on(window, 'gamepadconnected', this._padConnected);
      this._on(window, 'gamepaddisconnected', this._padDisconnected);
      this.padTimer = setInterval(() => this._pollPads(), GAMEPAD_POLL_MS);
      return;
    }
    this._on(window, 'keydown', this._keydown, true);
    this._on(window, 'keyup', this._keyup, true);
    this._on(window, 'blur', this.releaseAll);
    this._on(this.el, 'mousemove', this._mousemove);
    this._on(this.el, 'mousedown', this._mousebutton);
    this._on(this.el, 'mouseup', this._mousebutton);
    this._on(this.el, 'wheel', this._wheel, { passive: false });
    this._on(this.el, 'contextmenu', (e) => e.preventDefault());
    this._on(this.el, 'touchstart', this._touch, { passive: false });
    this._on(this.el, 'touchmove', this._touch, { passive: false });
    this._on(this.el, 'touchend', this._touch, { passive: false });
    this._on(window, 'gamepadconnected', this._padConnected);
    this._on(window, 'gamepaddisconnected', this._padDisconnected);
    this.padTimer = setInterval(() => this._pollPads(), GAMEPAD_POLL_MS);
  }

  detach() {
    for (const [t, type, h, opts] of this.listeners) t.removeEventListener(type, h, opts);
    this.listeners = [];
    clearInterval(this.padTimer);
    this.enabled = false;
  }

  releaseAll() {
    for (const ks of this.pressed.values()) this.send(`ku,${ks}`);
    this.pressed.clear();
    this.send('kr');
  }

  // ---------------------------------------------------------------- keyboard
  _keydown(e) {
    if (e.isComposing) return;
    const ks = keysymFor(e);
    if (ks === null) return;
    e.preventDefault();
    if (this.pressed.get(e.code) === ks && e.repeat) {
      this.send(`kd,${ks}`);          // autorepeat
      return;
    }
    this.pressed.set(e.code || e.key, ks);
    this.send(`kd,${ks}`);
  }

  _keyup(e) {
    const id = e.code || e.key;
    const ks = this.pressed.has(id) ? this.pressed.get(id) : keysymFor(e);
    this.pressed.delete(id);
    if (ks === null) return;
    e.preventDefault();
    this.send(`ku,${ks}`);
  }

  typeText(text) { this.send(`co,end,${text}`); }

  // ---------------------------------------------------------------- pointer
  _pos(e) {
    const r = this.el.getBoundingClientRect();
    const [sw, sh] = this.streamSize();
    return toStreamCoords(e.clientX - r.left, e.clientY - r.top, r.width, r.height, sw, sh);
  }

  _mousemove(e) {
    if (document.pointerLockElement === this.el) {
      this.send(mouseMessage(true, e.movementX, e.movementY, this.mask));
    } else {
      const [x, y] = this._pos(e);
      this.send(mouseMessage(false, x, y, this.mask));
    }
  }

  _mousebutton(e) {
    e.preventDefault();
    const bit = buttonBit(e.button);
    if (e.type === 'mousedown') this.mask |= bit; else this.mask &= ~bit;
    if (document.pointerLockElement === this.el) {
      this.send(mouseMessage(true, 0, 0, this.mask));
    } else {
      const [x, y] = this._pos(e);
      this.send(mouseMessage(false, x, y, this.mask));
    }
  }

  _wheelPulse(bit, magnitude) {
    magnitude = Math.max(1, Math.min(WHEEL_MAX_MAGNITUDE, Math.round(magnitude)));
    this.send(mouseMessage(true, 0, 0, this.mask | bit, magnitude));
    setTimeout(() => this.send(mouseMessage(true, 0, 0, this.mask & ~bit, magnitude)), 10);
  }

  _wheel(e) {
    e.preventDefault();
    if (e.deltaY) {
      const d = Math.abs(Math.trunc(e.deltaY)) || 1;
      this.smallestWheel = Math.min(this.smallestWheel, d);
      this._wheelPulse(e.deltaY < 0 ? MASK_WHEEL_UP : MASK_WHEEL_DOWN, Math.floor(d / this.smallestWheel));
    }
    if (e.deltaX) {
      this._wheelPulse(e.deltaX < 0 ? MASK_WHEEL_LEFT : MASK_WHEEL_RIGHT, Math.abs(e.deltaX) / 100);
    }
  }

  // Trackpad mode: one finger moves the pointer relatively, a short tap clicks,
  // two fingers scroll (handled below).
  _trackpad(e) {
    const t = e.changedTouches[0];
    const now = performance.now();
    if (e.type === 'touchstart') {
      this._tp = { x: t.clientX, y: t.clientY, x0: t.clientX, y0: t.clientY, t0: now };
    } else if (e.type === 'touchmove' && this._tp) {
      const dx = (t.clientX - this._tp.x) * 1.5;
      const dy = (t.clientY - this._tp.y) * 1.5;
      this._tp.x = t.clientX;
      this._tp.y = t.clientY;
      if (dx || dy) this.send(mouseMessage(true, dx, dy, this.mask));
    } else if (e.type === 'touchend' && this._tp) {
      const moved = Math.hypot(t.clientX - this._tp.x0, t.clientY - this._tp.y0);
      if (now - this._tp.t0 < 200 && moved < 8) {
        this.send(mouseMessage(true, 0, 0, this.mask | 1));
        this.send(mouseMessage(true, 0, 0, this.mask & ~1));
      }
      this._tp = null;
    }
  }

  // Single finger = left-button drag, two fingers = vertical scroll.
  _touch(e) {
    e.preventDefault();
    const t = e.touches;
    if (this.trackpad && (t.length <= 1)) {
      this._trackpad(e);
      return;
    }
    if (t.length === 1) {
      const [x, y] = this._pos(t[0]);
      const down = e.type !== 'touchend';
      const mask = down ? (this.mask | 1) : (this.mask & ~1);
      this.mask = mask;
      this.send(mouseMessage(false, x, y, mask));
      this._lastTouchY = null;
    } else if (t.length === 2) {
      const y = (t[0].clientY + t[1].clientY) / 2;
      if (this._lastTouchY != null && Math.abs(y - this._lastTouchY) > 12) {
        this._wheelPulse(y < this._lastTouchY ? MASK_WHEEL_DOWN : MASK_WHEEL_UP, 1);
        this._lastTouchY = y;
      } else if (this._lastTouchY == null) {
        this._lastTouchY = y;
      }
    } else if (e.type === 'touchend' && this.mask & 1) {
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
