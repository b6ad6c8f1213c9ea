"""The planner's host worker pool (csrc/ba_plan.cpp PlanPool) under back-to-back
parallel phases: every task exactly once, no deadlock, task exceptions
reach the caller (tests/cpp/plan_pool_test.cpp, built by the Makefile).
Runs on the CPU; 8 pool threads whatever the host reports."""
import os
import subprocess

import pytest

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "plan_pool_test")


@pytest.mark.skipif(not os.path.exists(EXE), reason="tests/cpp/plan_pool_test not built (make)")
def test_plan_pool_stress():
    env = dict(os.environ, SFM_PLAN_THREADS="8")
    r = subprocess.run([EXE, "20000"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 bad, exception caught" in r.stdout
