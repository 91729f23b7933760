// KeyboardEvent -> X11 keysym (the `kd,<keysym>` / `ku,<keysym>` messages).
// Named keys use the X11 keysymdef.h values; printable characters map to their
// Latin-1 keysym or to the Unicode keysym plane (0x01000000 | codepoint).

const NAMED = {
  Backspace: 0xff08, Tab: 0xff09, Enter: 0xff0d, Escape: 0xff1b, Delete: 0xffff, Home: 0xff50,
  ArrowLeft: 0xff51, ArrowUp: 0xff52, ArrowRight: 0xff53, ArrowDown: 0xff54, PageUp: 0xff55, PageDown: 0xff56,
  End: 0xff57, Insert: 0xff63, Pause: 0xff13, ScrollLock: 0xff14, PrintScreen: 0xff61, ContextMenu: 0xff67,
  NumLock: 0xff7f, CapsLock: 0xffe5, AltGraph: 0xfe03, Clear: 0xff0b, Help: 0xff6a, Cancel: 0xff69,
  Select: 0xff60, Execute: 0xff62, Find: 0xff68, Undo: 0xff65, Redo: 0xff66, Hiragana: 0xff25, Katakana: 0xff26,
  HiraganaKatakana: 0xff27, KanjiMode: 0xff21, Convert: 0xff23, NonConvert: 0xff22, Eisu: 0xff2f,
  HangulMode: 0xff31, HanjaMode: 0xff34, AudioVolumeMute: 0x1008ff12, AudioVolumeDown: 0x1008ff11,
  AudioVolumeUp: 0x1008ff13, MediaPlayPause: 0x1008ff14, MediaStop: 0x1008ff15, MediaTrackPrevious: 0x1008ff16,
  MediaTrackNext: 0x1008ff17, BrowserBack: 0x1008ff26, BrowserForward: 0x1008ff27, BrowserRefresh: 0x1008ff29,
};

// Keys whose left/right variant is only visible in KeyboardEvent.code.
const BY_CODE = {
  ShiftLeft: 0xffe1, ShiftRight: 0xffe2, ControlLeft: 0xffe3, ControlRight: 0xffe4, AltLeft: 0xffe9,
  AltRight: 0xffea, MetaLeft: 0xffeb, MetaRight: 0xffec, OSLeft: 0xffeb, OSRight: 0xffec,
  NumpadEnter: 0xff8d,
};

const NUMPAD = {
  Numpad0: [0xffb0, 0xff9e], Numpad1: [0xffb1, 0xff9c], Numpad2: [0xffb2, 0xff99], Numpad3: [0xffb3, 0xff9b],
  Numpad4: [0xffb4, 0xff96], Numpad5: [0xffb5, 0xff9d], Numpad6: [0xffb6, 0xff98], Numpad7: [0xffb7, 0xff95],
  Numpad8: [0xffb8, 0xff97], Numpad9: [0xffb9, 0xff9a], NumpadDecimal: [0xffae, 0xff9f],
  NumpadAdd: [0xffab, 0xffab], NumpadSubtract: [0xffad, 0xffad], NumpadMultiply: [0xffaa, 0xffaa],
  NumpadDivide: [0xffaf, 0xffaf],
};

export function charToKeysym(ch) {
  const cp = ch.codePointAt(0);
  if (cp === undefined) return null;
  if ((cp >= 0x20 && cp <= 0x7e) || (cp >= 0xa0 && cp <= 0xff)) return cp;
  if (cp === 0x0a || cp === 0x0d) return 0xff0d;
  if (cp === 0x09) return 0xff09;
  return (0x01000000 | cp) >>> 0;
}

// Returns the keysym for a KeyboardEvent-like {key, code, getModifierState?}, or null.
export function keysymFor(ev) {
  const code = ev.code || '';
  if (code in BY_CODE) return BY_CODE[code];
  if (code in NUMPAD) {
    const numLock = ev.getModifierState ? ev.getModifierState('NumLock') : true;
    const [on, off] = NUMPAD[code];
    return numLock ? on : off;
  }
  const key = ev.key;
  if (!key || key === 'Unidentified' || key === 'Dead' || key === 'Process') return null;
  if (key in NAMED) return NAMED[key];
  const f = /^F([0-9]{1,2})$/.exec(key);
  if (f) {
    const n = parseInt(f[1], 10);
    if (n >= 1 && n <= 35) return 0xffbe + n - 1;
  }
  if (key === 'Shift') return 0xffe1;
  if (key === 'Control') return 0xffe3;
  if (key === 'Alt') return 0xffe9;
  if (key === 'Meta' || key === 'OS') return 0xffeb;
  if ([...key].length === 1) return charToKeysym(key);
  return null;
}

export const MODIFIER_KEYSYMS = new Set([0xffe1, 0xffe2, 0xffe3, 0xffe4, 0xffe9, 0xffea, 0xffeb, 0xffec, 0xfe03]);
