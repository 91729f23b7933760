"""``selkies`` import name of the MI355X build (reference pyproject.toml:58-59,
src/selkies/).

Code written against the reference keeps its imports: ``selkies.settings``,
``selkies.input_handler``, ``selkies.selkies``, ``selkies.webrtc`` and
``selkies.legacy.*`` resolve to the modules of :mod:`selkies_gstreamer_amd` that
implement them. The alias is a module finder, so nothing heavy is imported until
a submodule is asked for.
"""
from __future__ import annotations

import importlib
import importlib.abc
import importlib.util
import sys

# reference module -> implementing module
ALIASES = {
    "selkies.settings": "selkies_gstreamer_amd.server.settings",
    "selkies.input_handler": "selkies_gstreamer_amd.server.input",
    "selkies.selkies": "selkies_gstreamer_amd.server.app",
    "selkies.server_keysym_map": "selkies_gstreamer_amd.server.input",
    "selkies.webrtc": "selkies_gstreamer_amd.webrtc",
    "selkies.legacy": "selkies_gstreamer_amd.legacy",
    "selkies.legacy.gstwebrtc_app": "selkies_gstreamer_amd.legacy.webrtc_app",
    "selkies.legacy.webrtc": "selkies_gstreamer_amd.legacy.webrtc_app",
    "selkies.legacy.webrtc_signalling": "selkies_gstreamer_amd.legacy.signalling_client",
    "selkies.legacy.signalling_web": "selkies_gstreamer_amd.legacy.signalling",
    "selkies.legacy.webrtc_input": "selkies_gstreamer_amd.server.input",
    "selkies.legacy.gamepad": "selkies_gstreamer_amd.server.gamepad",
    "selkies.legacy.metrics": "selkies_gstreamer_amd.server.metrics",
    "selkies.legacy.gpu_monitor": "selkies_gstreamer_amd.server.stats",
    "selkies.legacy.system_monitor": "selkies_gstreamer_amd.server.stats",
    "selkies.legacy.resize": "selkies_gstreamer_amd.server.display",
}


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target: str):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        real = ALIASES.get(fullname)
        if real is None and fullname.startswith(("selkies.webrtc.", "selkies.legacy.")):
            real = "selkies_gstreamer_amd." + fullname.split(".", 1)[1]
        if real is None:
            return None
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())


def __getattr__(name):
    full = f"selkies.{name}"
    if full in ALIASES:
        return importlib.import_module(full)
    raise AttributeError(name)
