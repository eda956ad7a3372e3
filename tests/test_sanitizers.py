"""Host AddressSanitizer + UndefinedBehaviorSanitizer run: the CPU restatement
(oracle/) and the library's host-only sources (csrc/cg_track.cpp tracker, csrc/cg_synth.c
synthetic frames) built with -fsanitize=address,undefined -fno-sanitize-recover=all
(`make -C oracle asan`) and driven by tests/sanitize/asan_driver.cpp over every size class,
edge clouds, the three parameter profiles, both voxel orders, the re-crop, the node's
tracking with full / short / failed colour responses and the tracker's C-ABI. Any report
aborts the driver. CPU only."""
import os
import subprocess

import cones_perception_amd as cp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)
    blobs = []
    for prof in ("simulation", "our", "fsai"):
        p = tmp_path / f"{prof}.params"
        p.write_bytes(bytes(cp.load_params(prof)))
        blobs.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "asan", "asan_driver"), *blobs],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "sanitizers clean" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
