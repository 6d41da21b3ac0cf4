"""Auxiliary subsystems: roctx ranges are no-ops without DLS_ROCTX, the
round watchdog turns a hang into a non-zero exit with the stacks on stderr, and the
self-launcher stops the other ranks when one fails (clean job abort)."""

import os
import subprocess
import sys
import textwrap
import time

from distributed_learning_simulator_amd.utils import tracing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trace_is_noop_without_env():
    with tracing.trace("x"):
        pass


def test_watchdog_quiet_when_in_time():
    fired = []
    with tracing.Watchdog(5.0, "quick", on_fire=lambda: fired.append(1)):
        time.sleep(0.01)
    time.sleep(0.05)
    assert not fired


def test_watchdog_aborts_hung_round():
    code = textwrap.dedent("""
        import time
        from distributed_learning_simulator_amd.utils.tracing import Watchdog
        with Watchdog(0.5, "round 7"):
            time.sleep(30)
    """)
    t = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == tracing.WATCHDOG_EXIT
    assert "[watchdog] round 7 exceeded" in r.stderr
    assert "in <module>" in r.stderr  # the hung thread's stack (faulthandler)
    assert time.perf_counter() - t < 20


def test_round_timeout_from_config_and_env(monkeypatch):
    class C:
        extra = {"round_timeout_s": 12}

    assert tracing.round_timeout(C()) == 12.0
    monkeypatch.setenv("DLS_ROUND_TIMEOUT", "3")
    assert tracing.round_timeout(C()) == 3.0


def test_launcher_stops_peers_when_a_rank_fails(tmp_path):
    script = tmp_path / "ranks.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            time.sleep(0.5)
            sys.exit(3)
        time.sleep(120)  # rank 0 would block in its next collective
    """))
    code = (f"import sys; from distributed_learning_simulator_amd.parallel import launch; "
            f"sys.exit(launch.spawn_ranks(2, argv=[], script={str(script)!r}))")
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "DLS_LAUNCHED_RANK"):
        env.pop(k, None)
    t = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode == 3
    assert time.perf_counter() - t < 30
