// Sidebar dashboard: screen / audio / stats / sharing / gamepad / input panels
// on top of the basic controls in index.html, with the server's ui_* settings
// deciding what is shown.
//
// Parity target: addons/selkies-dashboard (sidebar sections video, audio,
// screen, stats, clipboard, files, apps, sharing, gamepads, fullscreen, gaming
// mode, trackpad, keyboard button, soft buttons; each behind a
// ui_sidebar_show_* setting, settings.py:36-108). Pure helpers are exported for
// the node unit tests; the DOM code is plain ES modules without a framework.
import { TouchGamepad } from './touch-gamepad.js';
import { translator, pickLanguage, isRtl, LANGUAGE_NAMES } from './i18n.js';
import { parseCatalog, filterApps, appCommand, loadInstalled, updateInstalled, saveInstalled } from './apps.js';

// ui_sidebar_show_* flag -> data-section names it controls.
export const SECTION_FLAGS = {
  ui_sidebar_show_video_settings: ['video'],
  ui_sidebar_show_audio_settings: ['audio'],
  ui_sidebar_show_screen_settings: ['screen'],
  ui_sidebar_show_stats: ['stats'],
  ui_sidebar_show_clipboard: ['clipboard'],
  ui_sidebar_show_files: ['files'],
  ui_sidebar_show_apps: ['apps'],
  ui_sidebar_show_sharing: ['sharing'],
  ui_sidebar_show_gamepads: ['gamepads'],
  ui_sidebar_show_fullscreen: ['fullscreen'],
  ui_sidebar_show_gaming_mode: ['gaming'],
  ui_sidebar_show_trackpad: ['trackpad'],
  ui_sidebar_show_keyboard_button: ['keyboard'],
  ui_sidebar_show_soft_buttons: ['softkeys'],
};

const flag = (st, name, dflt = true) => {
  const d = st && st[name];
  if (d == null) return dflt;
  const v = typeof d === 'object' && 'value' in d ? d.value : d;
  return v === true || v === 'true' || v === 1;
};

// Sections to show for a server settings payload (missing flags default to shown).
export function visibleSections(st) {
  const out = new Set();
  if (!flag(st, 'ui_show_sidebar')) return out;
  for (const [name, sections] of Object.entries(SECTION_FLAGS)) {
    if (flag(st, name)) sections.forEach((s) => out.add(s));
  }
  if (!flag(st, 'audio_enabled')) out.delete('audio');
  if (!flag(st, 'clipboard_enabled')) out.delete('clipboard');
  if (!flag(st, 'gamepad_enabled')) out.delete('gamepads');
  if (!flag(st, 'command_enabled')) out.delete('apps');
  const ft = st && st.file_transfers;
  const transfers = ft == null ? 'upload,download' : String(typeof ft === 'object' && 'value' in ft ? ft.value : ft);
  if (!transfers.includes('upload')) out.delete('files');
  return out;
}

// Share links of the current page: view-only and player 2-4 (gamepad-only) URLs.
export function sharingLinks(href, st, t = translator('en')) {
  const base = href.split('#')[0];
  const links = [];
  if (!flag(st, 'enable_sharing')) return links;
  if (flag(st, 'enable_shared')) links.push({ label: t('sharing.viewOnly'), url: `${base}#shared` });
  for (const n of [2, 3, 4]) {
    if (flag(st, `enable_player${n}`)) links.push({ label: t('sharing.player', { n }), url: `${base}#player${n}` });
  }
  return links;
}

// Page hash -> display / sharing role.
export function parseRole(hash) {
  const h = hash.replace(/^#/, '');
  const d = /^display2(?:-(left|right|up|down))?$/.exec(h);
  if (d) return { id: 'display2', position: d[1] || 'right', shared: false, player: 1 };
  const p = /^player([234])$/.exec(h);
  if (p) return { id: 'primary', position: 'right', shared: true, player: parseInt(p[1], 10) };
  return { id: 'primary', position: 'right', shared: h === 'shared', player: h === 'shared' ? 0 : 1 };
}

// X11 keysyms of the soft buttons (sent as kd/ku pairs; combos press in order, release reversed).
export const SOFT_KEYS = {
  Esc: [0xff1b], Tab: [0xff09], Ctrl: [0xffe3], Alt: [0xffe9], Super: [0xffeb], F11: [0xffc8],
  'Ctrl+Alt+Del': [0xffe3, 0xffe9, 0xffff], 'Alt+Tab': [0xffe9, 0xff09], 'Ctrl+C': [0xffe3, 0x63],
  'Ctrl+V': [0xffe3, 0x76],
};

export function softKeyMessages(name) {
  const keys = SOFT_KEYS[name];
  if (!keys) return [];
  return [...keys.map((k) => `kd,${k}`), ...keys.slice().reverse().map((k) => `ku,${k}`)];
}

// Fixed-length history for the stats sparklines.
export class Ring {
  constructor(n = 60) { this.n = n; this.v = []; }
  push(x) { if (x == null || Number.isNaN(x)) return; this.v.push(+x); if (this.v.length > this.n) this.v.shift(); }
  max() { return this.v.length ? Math.max(...this.v) : 0; }
  last() { return this.v.length ? this.v[this.v.length - 1] : null; }
}

// Polyline points of a sparkline of `ring` in a w x h box (y up, min 0).
export function sparkPoints(ring, w, h) {
  const top = Math.max(ring.max(), 1e-9);
  const n = ring.v.length;
  return ring.v.map((x, i) => [n > 1 ? (i * (w - 1)) / (ring.n - 1) : 0, h - 1 - (x / top) * (h - 2)]);
}

// Dashboard layouts: the reference ships three dashboards over one client core
// (addons/selkies-dashboard: left sidebar; addons/selkies-dashboard-zinc: right
// side menu of collapsible panels; addons/selkies-dashboard-wish: top menu bar).
// Here they are three layouts of the same panels, picked by `?ui=<name>` or the
// `ui_dashboard` server setting; index.html styles `body.ui-<name>`.
export const LAYOUTS = {
  selkies: { side: 'left', collapsible: false, menu: 'sidebar' },
  zinc: { side: 'right', collapsible: true, menu: 'side-menu' },
  wish: { side: 'top', collapsible: true, menu: 'top-menu' },
};

export function pickLayout(search, st) {
  const m = /[?&]ui=([a-z]+)/.exec(search || '');
  if (m && m[1] in LAYOUTS) return m[1];
  const d = st && st.ui_dashboard;
  const v = d == null ? null : (typeof d === 'object' && 'value' in d ? d.value : d);
  return v in LAYOUTS ? v : 'selkies';
}

// Gamepad visualiser (reference GamepadVisualizer.jsx): standard-mapping pad as
// a list of shapes: buttons (filled when pressed, opacity = analog value) and the
// two sticks with their deflection. Rendered to SVG by padSvg().
const PAD_BUTTONS = [   // standard mapping index -> [x, y, r]
  [170, 62, 9], [186, 46, 9], [154, 46, 9], [170, 30, 9],      // A B X Y
  [40, 8, 7], [160, 8, 7], [40, 0, 6], [160, 0, 6],            // LB RB LT RT
  [84, 46, 5], [116, 46, 5], [72, 84, 10], [128, 84, 10],      // back start L3 R3
  [30, 30, 6], [30, 62, 6], [14, 46, 6], [46, 46, 6], [100, 30, 6],   // d-pad up/down/left/right, guide
];

export function padShapes(pad) {
  const shapes = [];
  const btn = (i) => (pad.buttons && pad.buttons[i]) || { pressed: false, value: 0 };
  PAD_BUTTONS.forEach(([x, y, r], i) => {
    const b = btn(i);
    const v = typeof b === 'number' ? b : (b.value || (b.pressed ? 1 : 0));
    shapes.push({ kind: 'button', index: i, x, y, r, on: v > 0.1 || !!b.pressed, value: Math.min(1, Math.max(0, v)) });
  });
  const ax = pad.axes || [];
  [[72, 84, 0, 1], [128, 84, 2, 3]].forEach(([cx, cy, ix, iy], k) => {
    const dx = Math.max(-1, Math.min(1, ax[ix] || 0)), dy = Math.max(-1, Math.min(1, ax[iy] || 0));
    shapes.push({ kind: 'stick', index: k, x: cx + dx * 8, y: cy + dy * 8, r: 6 });
  });
  return shapes;
}

export function padSvg(pad) {
  const body = padShapes(pad).map((s) => (s.kind === 'button'
    ? `<circle cx="${s.x}" cy="${s.y}" r="${s.r}" fill="${s.on ? '#7cf' : 'none'}" fill-opacity="${s.on ? Math.max(0.3, s.value) : 0}" stroke="#9ab"/>`
    : `<circle cx="${s.x.toFixed(1)}" cy="${s.y.toFixed(1)}" r="${s.r}" fill="#fc6"/>`)).join('');
  return `<svg xmlns="http://www.w3.org/2000/svg" viewBox="0 -8 200 110" width="200" height="110">${body}</svg>`;
}

// System monitor gauges from the server's system_stats / gpu_stats / network_stats
// messages (server/stats.py; reference system-monitoring.tsx): fractions 0..1.
export function monitorGauges(stats, t = translator('en')) {
  const frac = (x) => (x == null || Number.isNaN(+x) ? null : Math.max(0, Math.min(1, +x)));
  return [
    { key: 'cpu', label: 'CPU', value: stats.cpu == null ? null : frac(stats.cpu / 100) },
    { key: 'mem', label: t('monitor.memory'), value: frac(stats.mem) },
    { key: 'gpu', label: 'GPU', value: frac(stats.gpu) },
    { key: 'vram', label: 'VRAM', value: frac(stats.vram) },
  ];
}

// Keyboard shortcuts panel (reference shortcuts-menu.tsx): label -> soft key combo.
export const SHORTCUTS = [
  ['shortcuts.menu', 'Ctrl+Shift+M'], ['shortcuts.fullscreen', 'Ctrl+Shift+F'], ['shortcuts.pointer', 'Ctrl+Shift+click'],
];

// Headings of the static index.html blocks -> (section, translation key).
export const STATIC_HEADS = {
  Video: ['video', 'section.video'], Audio: ['audio', 'section.audio'], Screen: ['fullscreen', 'section.screen'],
  Clipboard: ['clipboard', 'section.clipboard'], Files: ['files', 'section.files'], Stats: ['stats', 'section.stats'],
};

export const DPI_CHOICES = [96, 120, 144, 168, 192, 216, 240, 264, 288];
export const AUDIO_BITRATES = [64000, 128000, 265000, 320000];

// -------------------------------------------------------------------- DOM
const STAT_KEYS = [['fps', 'fps'], ['mbps', 'Mbit/s'], ['rtt', 'ms'], ['cpu', 'cpu %'], ['gpu', 'gpu']];

export class Dashboard {
  constructor(client, doc = document) {
    this.c = client;
    this.doc = doc;
    const store = typeof localStorage !== 'undefined' ? localStorage : null;
    const saved = store && store.getItem('selkiesLang');
    const prefs = typeof navigator !== 'undefined' ? (navigator.languages || [navigator.language]) : [];
    this.t = translator(pickLanguage(typeof location !== 'undefined' ? location.search : '', [saved, ...prefs]));
    this.rings = Object.fromEntries(STAT_KEYS.map(([k]) => [k, new Ring(60)]));
    this.touchPad = null;
  }

  el(tag, attrs = {}, children = []) {
    const e = this.doc.createElement(tag);
    for (const [k, v] of Object.entries(attrs)) {
      if (k === 'text') e.textContent = v; else if (k.startsWith('on')) e[k] = v; else e.setAttribute(k, v);
    }
    for (const ch of children) e.appendChild(ch);
    return e;
  }

  section(name, title, children) {
    return this.el('div', { 'data-section': name }, [this.el('h3', { text: title }), ...children]);
  }

  setLayout(name) {
    const body = this.doc.body;
    for (const n of Object.keys(LAYOUTS)) body.classList.remove(`ui-${n}`);
    body.classList.add(`ui-${name}`);
    this.layout = name;
  }

  // zinc / wish: a click on a panel heading folds the panel
  _collapsible(sb) {
    for (const h of sb.querySelectorAll('h3')) {
      h.onclick = () => {
        if (!LAYOUTS[this.layout || 'selkies'].collapsible) return;
        const folded = h.classList.toggle('folded');
        for (let n = h.nextElementSibling; n && n.tagName !== 'H3' && !(n.dataset && n.dataset.section); n = n.nextElementSibling) {
          n.classList.toggle('fold-hidden', folded);
        }
        const sec = h.parentElement && h.parentElement.dataset && h.parentElement.dataset.section ? h.parentElement : null;
        if (sec) for (const n of sec.children) if (n !== h) n.classList.toggle('fold-hidden', folded);
      };
    }
  }

  build() {
    const sb = this.doc.getElementById('sidebar');
    const s = this.c.settings;
    this.setLayout(pickLayout(typeof location !== 'undefined' ? location.search : '', this.c.serverSettings));
    // screen
    const mw = this.el('input', { type: 'number', min: '320', max: '7680', step: '2', value: s.manual_width || 1920,
      style: 'width:70px' });
    const mh = this.el('input', { type: 'number', min: '240', max: '4320', step: '2', value: s.manual_height || 1080,
      style: 'width:70px' });
    const manual = this.el('input', { type: 'checkbox' });
    manual.checked = !!s.is_manual_resolution_mode;
    const applyRes = () => {
      const w = parseInt(mw.value, 10) & ~1;
      const h = parseInt(mh.value, 10) & ~1;
      this.c.settings.manual_width = w;
      this.c.settings.manual_height = h;
      this.c.updateSetting('is_manual_resolution_mode', manual.checked);
      if (manual.checked) this.c.sendText(`r,${w}x${h},${this.c.display.id}`);
    };
    manual.onchange = applyRes;
    const dpi = this.el('select', {}, DPI_CHOICES.map((d) => this.el('option', { value: d, text: `${d} dpi` })));
    dpi.value = s.scaling_dpi || 96;
    dpi.onchange = () => this.c.updateSetting('scaling_dpi', parseInt(dpi.value, 10));
    const css = this.el('input', { type: 'checkbox' });
    css.checked = !!s.use_css_scaling;
    css.onchange = () => this.c.updateSetting('use_css_scaling', css.checked);
    const t = this.t;
    if (this.doc.documentElement) {
      this.doc.documentElement.lang = t.lang;
      this.doc.documentElement.dir = isRtl(t.lang) ? 'rtl' : 'ltr';
    }
    sb.appendChild(this.section('screen', t('section.screen'), [
      this.el('label', { text: t('screen.manual') }, [manual]),
      this.el('label', {}, [mw, this.el('span', { text: 'x' }), mh,
        this.el('button', { text: t('screen.apply'), onclick: applyRes })]),
      this.el('label', { text: t('screen.scaling') }, [dpi]),
      this.el('label', { text: t('screen.css') }, [css]),
    ]));
    // audio bitrate
    const ab = this.el('select', {}, AUDIO_BITRATES.map((b) => this.el('option', { value: b, text: `${b / 1000} kbit/s` })));
    ab.value = s.audio_bitrate || 320000;
    ab.onchange = () => this.c.updateSetting('audio_bitrate', parseInt(ab.value, 10));
    this.audioBitrate = ab;
    sb.appendChild(this.section('audio', t('section.audio'), [this.el('label', { text: t('audio.bitrate') }, [ab])]));
    // input
    const gaming = this.el('input', { type: 'checkbox' });
    gaming.onchange = () => {
      if (gaming.checked) { this.c.input.requestPointerLock(); this.c.canvas.style.cursor = 'none'; } else {
        if (this.doc.exitPointerLock) this.doc.exitPointerLock();
        this.c.canvas.style.cursor = '';
      }
    };
    const tp = this.el('input', { type: 'checkbox' });
    tp.onchange = () => { this.c.input.trackpad = tp.checked; };
    const kb = this.el('input', { type: 'text', 'aria-label': 'keyboard', autocapitalize: 'off', autocomplete: 'off',
      style: 'position:absolute;left:-1000px;opacity:0' });
    kb.oninput = () => { if (kb.value) { this.c.input.typeText(kb.value); kb.value = ''; } };
    sb.appendChild(this.section('gaming', t('section.input'), [this.el('label', { text: t('input.gaming') }, [gaming])]));
    sb.appendChild(this.section('trackpad', '', [this.el('label', { text: t('input.trackpad') }, [tp])]));
    sb.appendChild(this.section('keyboard', '', [kb, this.el('button', { text: t('input.keyboard'),
      onclick: () => kb.focus() })]));
    sb.appendChild(this.section('softkeys', t('section.keys'), Object.keys(SOFT_KEYS).map((name) => this.el('button', {
      text: name, onclick: () => softKeyMessages(name).forEach((m) => this.c.sendText(m)) }))));
    // apps: catalog with search + install / remove / update, and a free command line
    const cmd = this.el('input', { type: 'text', placeholder: t('apps.command'), style: 'width:150px' });
    this.appSearch = this.el('input', { type: 'search', placeholder: t('apps.search'), style: 'width:180px' });
    this.appList = this.el('div', { style: 'max-height:220px;overflow-y:auto' });
    this.appSearch.oninput = () => this.renderApps();
    sb.appendChild(this.section('apps', t('section.apps'), [this.appSearch, this.appList,
      this.el('label', {}, [cmd, this.el('button', { text: t('apps.run'),
        onclick: () => { if (cmd.value.trim()) this.c.sendText(`cmd,${cmd.value.trim()}`); } })])]));
    // files: the server's download directory listing (./files/) in a modal frame
    sb.appendChild(this.section('files', t('section.files'), [this.el('button', { text: t('files.open'),
      onclick: () => this.toggleFiles(true) })]));
    // sharing
    this.shareBox = this.el('div');
    sb.appendChild(this.section('sharing', t('section.sharing'), [this.shareBox]));
    // gamepads
    this.padBox = this.el('div', { style: 'white-space:pre;font:12px ui-monospace,monospace' });
    sb.appendChild(this.section('gamepads', t('section.gamepads'), [this.padBox, this.el('button', { text: t('gamepads.touch'),
      onclick: () => { if (!this.touchPad) this.touchPad = new TouchGamepad(); this.touchPad.toggle(); } })]));
    // stats sparklines
    this.sparks = {};
    const graphs = STAT_KEYS.map(([k, label]) => {
      const cv = this.el('canvas', { width: 120, height: 22 });
      const v = this.el('span', { text: '-' });
      this.sparks[k] = { cv, v };
      return this.el('label', { text: label }, [cv, v]);
    });
    sb.appendChild(this.section('stats', t('section.graphs'), graphs));
    // system monitor gauges
    this.gauges = {};
    const gaugeRows = monitorGauges({}, t).map((g) => {
      const bar = this.el('progress', { max: '100', value: '0', style: 'width:130px' });
      this.gauges[g.key] = bar;
      return this.el('label', { text: g.label }, [bar]);
    });
    sb.appendChild(this.section('stats', t('section.monitor'), gaugeRows));
    // gamepad visualiser
    this.padViz = this.el('div');
    sb.appendChild(this.section('gamepads', t('section.gamepads'), [this.padViz]));
    // shortcuts
    sb.appendChild(this.section('softkeys', t('section.shortcuts'), SHORTCUTS.map(([what, keys]) =>
      this.el('label', { text: t(what) }, [this.el('kbd', { text: keys })]))));
    // language
    const lang = this.el('select', {}, Object.entries(LANGUAGE_NAMES).map(([code, name]) =>
      this.el('option', { value: code, text: name })));
    lang.value = t.lang;
    lang.onchange = () => {
      if (typeof localStorage !== 'undefined') localStorage.setItem('selkiesLang', lang.value);
      if (typeof location !== 'undefined') location.reload();
    };
    sb.appendChild(this.el('div', { 'data-section-lang': '1' }, [this.el('h3', { text: t('section.language') }), lang]));
    this._collapsible(sb);
    // tag (and translate) the static sections of index.html
    for (const h of sb.querySelectorAll(':scope > h3')) {
      const m = STATIC_HEADS[h.textContent.trim()];
      if (m) {
        h.setAttribute('data-section-head', m[0]);
        h.textContent = t(m[1]);
      }
    }
    this.installed = loadInstalled(typeof localStorage !== 'undefined' ? localStorage : null);
    this.apps = [];
    this.timer = setInterval(() => this.tick(), 1000);
  }

  // Files modal: the server's ./files/ listing (download directory) in an iframe.
  toggleFiles(open) {
    if (!open) {
      if (this.filesModal) this.filesModal.remove();
      this.filesModal = null;
      return;
    }
    if (this.filesModal) return;
    const frame = this.el('iframe', { src: './files/', title: this.t('section.files'),
      style: 'width:100%;height:calc(100% - 32px);border:0;background:#fff' });
    this.filesModal = this.el('div', { style: 'position:fixed;inset:8%;z-index:5;background:#18181b;border-radius:6px;padding:4px' }, [
      this.el('button', { text: this.t('files.close'), onclick: () => this.toggleFiles(false) }), frame]);
    this.doc.body.appendChild(this.filesModal);
  }

  async loadApps(url) {
    try {
      const r = await fetch(url || './apps.json');
      if (!r.ok) throw new Error(`HTTP ${r.status}`);
      this.apps = parseCatalog(await r.json());
      this.appError = null;
    } catch (e) {
      this.apps = [];
      this.appError = this.t('apps.error');
    }
    this.renderApps();
  }

  appAction(action, name) {
    this.c.sendText(appCommand(action, name));
    this.installed = updateInstalled(this.installed, action, name);
    saveInstalled(typeof localStorage !== 'undefined' ? localStorage : null, this.installed);
    this.renderApps();
  }

  renderApps() {
    if (!this.appList) return;
    const t = this.t;
    const shown = filterApps(this.apps || [], this.appSearch ? this.appSearch.value : '');
    if (!shown.length) {
      this.appList.replaceChildren(this.el('div', { text: this.appError || t('apps.empty') }));
      return;
    }
    this.appList.replaceChildren(...shown.map((a) => {
      const have = (this.installed || []).includes(a.name);
      const acts = have ? ['update', 'remove'] : ['install'];
      return this.el('div', { title: a.description, style: 'display:flex;gap:6px;align-items:center' }, [
        this.el('span', { text: a.title, style: 'flex:1' }),
        ...acts.map((act) => this.el('button', { text: t(`apps.${act}`), onclick: () => this.appAction(act, a.name) })),
      ]);
    }));
  }

  apply(st) {
    this.setLayout(pickLayout(typeof location !== 'undefined' ? location.search : '', st));
    const vis = visibleSections(st);
    const sb = this.doc.getElementById('sidebar');
    for (const node of sb.querySelectorAll('[data-section]')) node.style.display = vis.has(node.dataset.section) ? '' : 'none';
    // static index.html blocks: hide a heading and the controls up to the next heading
    for (const h of sb.querySelectorAll('[data-section-head]')) {
      const show = vis.has(h.dataset.sectionHead);
      for (let n = h; n && (n === h || n.tagName !== 'H3'); n = n.nextElementSibling) {
        if (n.dataset && n.dataset.section) break;
        n.style.display = show ? '' : 'none';
      }
    }
    const toggle = this.doc.getElementById('toggle');
    if (toggle) toggle.style.display = vis.size ? '' : 'none';
    this.shareBox.replaceChildren(...sharingLinks(location.href, st, this.t).map((l) => this.el('div', {}, [
      this.el('a', { href: l.url, target: '_blank', text: l.label, style: 'color:#8cf' }),
      this.el('button', { text: this.t('sharing.copy'), onclick: () => navigator.clipboard && navigator.clipboard.writeText(l.url) }),
    ])));
    if (vis.has('apps') && !this.appsRequested) {
      this.appsRequested = true;
      const u = st.apps_catalog_url;
      this.loadApps(u && typeof u === 'object' && 'value' in u ? u.value : u);
    }
    const abDef = st.audio_bitrate;
    if (abDef && abDef.allowed) {
      this.audioBitrate.replaceChildren(...abDef.allowed.map((b) => this.el('option', { value: b, text: `${b / 1000} kbit/s` })));
      this.audioBitrate.value = this.c.settings.audio_bitrate;
    }
  }

  tick() {
    const st = this.c.stats;
    for (const [k] of STAT_KEYS) {
      const r = this.rings[k];
      let v = st[k];
      if (k === 'gpu' && v != null) v *= 100;
      r.push(v);
      const { cv, v: label } = this.sparks[k];
      label.textContent = r.last() == null ? '-' : `${Math.round(r.last() * 10) / 10}`;
      const g = cv.getContext && cv.getContext('2d');
      if (!g) continue;
      g.clearRect(0, 0, cv.width, cv.height);
      g.strokeStyle = '#7cf';
      g.beginPath();
      sparkPoints(r, cv.width, cv.height).forEach(([x, y], i) => (i ? g.lineTo(x, y) : g.moveTo(x, y)));
      g.stroke();
    }
    for (const g of monitorGauges(st, this.t)) {
      if (this.gauges && this.gauges[g.key]) this.gauges[g.key].value = g.value == null ? 0 : Math.round(g.value * 100);
    }
    if (navigator.getGamepads) {
      const pads = Array.from(navigator.getGamepads() || []).filter(Boolean);
      if (this.padViz) this.padViz.innerHTML = pads.length ? padSvg(pads[0]) : '';
      this.padBox.textContent = pads.length ? pads.map((p) => `${p.index}: ${p.id.slice(0, 28)}\n   `
        + `axes ${p.axes.map((a) => a.toFixed(1)).join(' ')}  buttons ${p.buttons.filter((b) => b.pressed).length}`)
        .join('\n') : this.t('gamepads.none');
    }
  }
}
