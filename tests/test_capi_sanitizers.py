"""CPU: the C ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "race detection /
sanitizers"). tests/native/build_asan.sh compiles capi.cpp, dit.cpp and vae_engine.cpp with host-only
-fsanitize=address,undefined (device code unchanged; GPU sanitizers are not available on this pool) and links
tests/native/capi_validation.cpp, which drives the argument, bind and shape validation of every engine and the
kernel entry points -- all refused before any device work, so no GPU is needed -- with leak detection on."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent


@pytest.mark.skipif(shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists(),
                    reason="hipcc not available")
def test_capi_validation_under_asan_ubsan():
    r = subprocess.run(["bash", str(HERE / "native" / "build_asan.sh")], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    exe = r.stdout.strip().splitlines()[-1]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "all checks passed" in r.stdout
