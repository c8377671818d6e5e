"""Host-code sanitizers: the C ABI's host-side graph planners (gine_graph_order_locality,
gine_graph_plan_windows, gine_graph_plan_window_slots) built with AddressSanitizer and
UndefinedBehaviorSanitizer on the host side only (`make hostasan` in csrc/: each
-fsanitize= behind -Xarch_host, device code untouched) and run on synthetic CSRs with edge
cases -- empty, single node, self loops only, isolated nodes, hubs, in-degree 33, an edge
budget below a node's degree -- every output checked against its contract
(tests/native/host_planner_asan.cpp).  No GPU call is made."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raincast-gnn_amd", "csrc")
BIN = os.path.join(CSRC, "build", "asan", "host_planner_asan")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc to build the sanitizer binary")
def test_host_planners_clean_under_asan_and_ubsan():
    subprocess.run(["make", "-s", "hostasan"], cwd=CSRC, check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([BIN], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host planner checks: ok" in r.stdout
