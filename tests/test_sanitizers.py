"""ASan+UBSan and TSan builds of the host C++ core, driven by the concurrency
stress program csrc/tests/stress.cc (concurrent HTTP/gRPC readers on shared
clients, injected 503s / disconnects / corruption, sliced reads, concurrent
uploads and listings against the in-process synthetic server).

SURVEY.md §4.5 / §5: the reference never runs a race detector and has real
races (Q3, Q14).  GPU code is not sanitized (GPU ASan is unavailable here)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(target):
    import fcntl

    jobs = str(min(8, os.cpu_count() or 4))
    # the parametrized cases share build targets: one make at a time (under
    # xdist two concurrent makes relinking one binary broke a run)
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".sanitizer_build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-C", ROOT, "-j", jobs, target], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("kind,env", [
    ("asan", {"ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "halt_on_error=1"}),
    ("tsan", {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"}),
])
def test_stress_under_sanitizer(kind, env):
    _build(f"build/{kind}/stress")
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([os.path.join(ROOT, "build", kind, "stress"), "2"], capture_output=True, text=True,
                       timeout=600, env=e)
    assert r.returncode == 0, f"{kind} stress failed (rc={r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-6000:]}"
    assert "stress: ok" in r.stdout
