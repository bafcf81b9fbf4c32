"""Native core under AddressSanitizer+UBSan and ThreadSanitizer (host code only).

Builds csrc/core/test_core.cpp -- concurrent membership registry traffic,
codec round trips + fuzzing, the ingest ring's host path -- with each
sanitizer and runs it (scripts/sanitize_core.sh).  SURVEY.md §5.2."""
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_core_under_asan_ubsan_and_tsan():
    proc = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_core.sh")], capture_output=True,
                          text=True, timeout=900)
    assert proc.returncode == 0, proc.stderr[-4000:]
    assert proc.stdout.split().count("ok") == 2, proc.stdout
