// Universal touch gamepad: an on-screen controller for touch devices that shows
// up to the page (and to lib/input.js, which forwards pads to the server's
// virtual Xbox 360 pads) as a regular standard-mapping Gamepad.
//
// Parity target: addons/universal-touch-gamepad/universalTouchGamepad.js of the
// reference, which injects a virtual device into navigator.getGamepads(). The
// geometry and state logic are pure functions (unit-tested under node); the DOM
// part only renders the controls and feeds touches into them.

// Standard mapping (https://w3c.github.io/gamepad/#remapping): button indices.
export const BUTTONS = {
  A: 0, B: 1, X: 2, Y: 3, LB: 4, RB: 5, LT: 6, RT: 7, SELECT: 8, START: 9,
  L3: 10, R3: 11, UP: 12, DOWN: 13, LEFT: 14, RIGHT: 15, HOME: 16,
};
export const NUM_BUTTONS = 17;
export const NUM_AXES = 4;

// Stick displacement (touch point relative to the stick centre) -> axis pair in
// [-1, 1], with a radial dead zone and clamping to the unit circle.
export function stickAxes(dx, dy, radius, deadzone = 0.12) {
  if (radius <= 0) return [0, 0];
  let x = dx / radius;
  let y = dy / radius;
  const m = Math.hypot(x, y);
  if (m < deadzone) return [0, 0];
  if (m > 1) { x /= m; y /= m; }
  // rescale so the dead zone edge maps to 0 (no jump when leaving it)
  const k = (Math.min(m, 1) - deadzone) / (1 - deadzone) / Math.min(m, 1);
  return [Math.round(x * k * 1000) / 1000, Math.round(y * k * 1000) / 1000];
}

// A d-pad touch selects up to two neighbouring directions (8-way).
export function dpadButtons(dx, dy, deadzone = 0.25, radius = 1) {
  const x = dx / radius;
  const y = dy / radius;
  const out = [];
  if (Math.hypot(x, y) < deadzone) return out;
  const a = Math.atan2(y, x) * 180 / Math.PI;   // 0 = right, 90 = down
  if (a > -67.5 && a < 67.5) out.push(BUTTONS.RIGHT);
  if (a > 22.5 && a < 157.5) out.push(BUTTONS.DOWN);
  if (a > 112.5 || a < -112.5) out.push(BUTTONS.LEFT);
  if (a > -157.5 && a < -22.5) out.push(BUTTONS.UP);
  return out;
}

// Gamepad-interface-shaped state object.
export class VirtualPad {
  constructor(index = 0, id = 'Selkies Universal Touch Gamepad (STANDARD GAMEPAD Vendor: 045e Product: 028e)') {
    this.id = id;
    this.index = index;
    this.connected = true;
    this.mapping = 'standard';
    this.axes = new Array(NUM_AXES).fill(0);
    this.buttons = Array.from({ length: NUM_BUTTONS }, () => ({ pressed: false, touched: false, value: 0 }));
    this.timestamp = 0;
  }

  setButton(i, pressed, value = pressed ? 1 : 0) {
    const b = this.buttons[i];
    if (b.pressed === pressed && b.value === value) return false;
    this.buttons[i] = { pressed, touched: pressed, value };
    this.timestamp = (typeof performance !== 'undefined' ? performance.now() : Date.now());
    return true;
  }

  setStick(which, x, y) {
    const o = which === 'left' ? 0 : 2;
    if (this.axes[o] === x && this.axes[o + 1] === y) return false;
    this.axes[o] = x;
    this.axes[o + 1] = y;
    this.timestamp = (typeof performance !== 'undefined' ? performance.now() : Date.now());
    return true;
  }

  setDpad(pressedList) {
    let changed = false;
    for (const i of [BUTTONS.UP, BUTTONS.DOWN, BUTTONS.LEFT, BUTTONS.RIGHT]) {
      changed = this.setButton(i, pressedList.includes(i)) || changed;
    }
    return changed;
  }
}

// navigator.getGamepads() that also reports the virtual pad (first free slot).
export function installGetGamepads(nav, pad) {
  const native = nav.getGamepads ? nav.getGamepads.bind(nav) : () => [];
  const patched = () => {
    const list = Array.from(native() || []);
    while (list.length <= pad.index) list.push(null);
    if (!list[pad.index]) list[pad.index] = pad;
    return list;
  };
  nav.getGamepads = patched;
  return () => { nav.getGamepads = native; };
}

export function freeIndex(nav) {
  const list = nav.getGamepads ? Array.from(nav.getGamepads() || []) : [];
  for (let i = 0; i < 4; i++) if (!list[i]) return i;
  return 3;
}

// -------------------------------------------------------------------- DOM controller
const LAYOUT = [
  // [label, button index, css position]
  ['A', BUTTONS.A, 'right:72px;bottom:40px'], ['B', BUTTONS.B, 'right:24px;bottom:88px'],
  ['X', BUTTONS.X, 'right:120px;bottom:88px'], ['Y', BUTTONS.Y, 'right:72px;bottom:136px'],
  ['LB', BUTTONS.LB, 'left:24px;top:24px'], ['RB', BUTTONS.RB, 'right:24px;top:24px'],
  ['LT', BUTTONS.LT, 'left:24px;top:76px'], ['RT', BUTTONS.RT, 'right:24px;top:76px'],
  ['SEL', BUTTONS.SELECT, 'left:calc(50% - 70px);bottom:24px'], ['START', BUTTONS.START, 'left:calc(50% + 14px);bottom:24px'],
  ['⌂', BUTTONS.HOME, 'left:calc(50% - 20px);bottom:70px'],
];

export class TouchGamepad {
  constructor(root = document.body, nav = navigator) {
    this.nav = nav;
    this.pad = new VirtualPad(freeIndex(nav));
    this.root = root;
    this.el = null;
    this.uninstall = null;
  }

  show() {
    if (this.el) return;
    this.uninstall = installGetGamepads(this.nav, this.pad);
    const el = document.createElement('div');
    el.id = 'touch-gamepad';
    el.style.cssText = 'position:fixed;inset:0;z-index:4;pointer-events:none;user-select:none;touch-action:none';
    const btnCss = 'position:absolute;pointer-events:auto;min-width:44px;height:44px;border-radius:22px;'
      + 'background:rgba(255,255,255,.18);color:#fff;display:flex;align-items:center;justify-content:center;'
      + 'font:bold 13px system-ui;border:1px solid rgba(255,255,255,.35)';
    for (const [label, idx, pos] of LAYOUT) {
      const b = document.createElement('div');
      b.textContent = label;
      b.style.cssText = `${btnCss};${pos}`;
      const set = (v) => (e) => { e.preventDefault(); this.pad.setButton(idx, v); };
      b.addEventListener('touchstart', set(true));
      b.addEventListener('touchend', set(false));
      b.addEventListener('touchcancel', set(false));
      el.appendChild(b);
    }
    el.appendChild(this._stick('left', 'left:40px;bottom:40px'));
    el.appendChild(this._stick('right', 'right:190px;bottom:150px'));
    el.appendChild(this._dpad('left:190px;bottom:40px'));
    this.root.appendChild(el);
    this.el = el;
    window.dispatchEvent(Object.assign(new Event('gamepadconnected'), { gamepad: this.pad }));
  }

  hide() {
    if (!this.el) return;
    this.el.remove();
    this.el = null;
    window.dispatchEvent(Object.assign(new Event('gamepaddisconnected'), { gamepad: this.pad }));
    if (this.uninstall) this.uninstall();
  }

  toggle() { if (this.el) this.hide(); else this.show(); }

  _zone(css, size) {
    const z = document.createElement('div');
    z.style.cssText = `position:absolute;pointer-events:auto;width:${size}px;height:${size}px;border-radius:50%;`
      + `background:rgba(255,255,255,.10);border:1px solid rgba(255,255,255,.3);${css}`;
    return z;
  }

  _track(zone, onMove, onEnd) {
    const move = (e) => {
      e.preventDefault();
      const t = e.targetTouches[0];
      if (!t) return;
      const r = zone.getBoundingClientRect();
      onMove(t.clientX - (r.left + r.width / 2), t.clientY - (r.top + r.height / 2), r.width / 2);
    };
    zone.addEventListener('touchstart', move);
    zone.addEventListener('touchmove', move);
    const end = (e) => { e.preventDefault(); onEnd(); };
    zone.addEventListener('touchend', end);
    zone.addEventListener('touchcancel', end);
  }

  _stick(which, css) {
    const z = this._zone(css, 120);
    this._track(z, (dx, dy, r) => { const [x, y] = stickAxes(dx, dy, r); this.pad.setStick(which, x, y); },
      () => this.pad.setStick(which, 0, 0));
    return z;
  }

  _dpad(css) {
    const z = this._zone(css, 110);
    z.style.borderRadius = '12px';
    this._track(z, (dx, dy, r) => this.pad.setDpad(dpadButtons(dx, dy, 0.25, r)), () => this.pad.setDpad([]));
    return z;
  }
}
