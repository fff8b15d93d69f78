"""The JavaScript host's CPU tests (tests/js/test_host.js) under Node."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_host():
    env = dict(os.environ)
    env.pop("VPT_HAVE_GPU", None)
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "test_host.js")], capture_output=True,
                       text=True, timeout=300, env=env)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
