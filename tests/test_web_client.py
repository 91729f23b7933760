"""Browser client (selkies_gstreamer_amd/web): every module parses under node and
the pure protocol / keysym / coordinate helpers pass their node unit tests."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
WEB = ROOT / "selkies_gstreamer_amd" / "web"
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


@pytest.mark.parametrize("path", sorted(p.relative_to(WEB).as_posix() for p in WEB.rglob("*.js")))
def test_module_syntax(path):
    r = subprocess.run([NODE, "--check", "--input-type=module"], input=(WEB / path).read_text(), capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr


def test_client_unit_tests():
    r = subprocess.run([NODE, str(ROOT / "tests" / "js" / "client_test.mjs")], capture_output=True, text=True,
                       timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "client tests ok" in r.stdout
    assert "i18n ok" in r.stdout and "apps ok" in r.stdout
    assert "webrtc client ok" in r.stdout and "codec strings ok" in r.stdout


def test_index_references_existing_modules():
    html = (WEB / "index.html").read_text()
    assert 'src="selkies-client.js"' in html
    for name in ("stream", "sidebar", "encoder", "framerate", "crf", "jpegq", "audio", "mic", "clip", "files", "stats"):
        assert f'id="{name}"' in html
