"""Host-code sanitizer run (no GPU): tests/asan builds the C ABI's host parts (OBJ/MTL ingestion
mcrt_objload.cpp, camera mcrt_camera.cpp, the host Bvh2 restatement mcrt_bvh.cpp) and the oracle with
AddressSanitizer + UndefinedBehaviorSanitizer, then loads an OBJ/MTL scene, traces it against brute
force, renders PT and BDPT frames, accumulates, denoises, tone-maps and builds a 30 k-triangle BVH
on 4 threads.  Any sanitizer finding aborts the program."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_code_under_asan_ubsan():
    d = os.path.join(HERE, "asan")
    subprocess.run(["make", "-C", d], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(d, "host_asan")], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host asan ok" in r.stdout
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
