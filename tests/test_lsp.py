"""The LSP transport (p1_amd/host/lsp.{hpp,cpp}, lspnet.{hpp,cpp}) against
the reference's own LSP test scenarios, restated in tests/lsp/lsp_scenarios.cpp
with the reference's parameters (client counts, message counts, EpochLimit /
EpochMillis / WindowSize, drop rates, timeouts):

  lsp1_test.go:201-335  Basic1-9, SendReceive1-3, Robust1-6
  lsp2_test.go:476-516  Window1-6
  lsp3_test.go:322-392  ServerSlowStart1-2, ServerClose1-2, ServerCloseConns1-2, ClientClose1-2
  lsp4_test.go:444-526  ServerFastClose1-3, ServerToClient1-3, ClientToServer1-3, RoundTrip1-3
  lsp5_test.go:193-203  VariableLengthMsgServer/Client

One process per scenario: the fault-injection knobs are process-global, as
in the reference (lspnet/staff.go)."""
import os
import subprocess

import pytest

from conftest import ROOT, host_bin

DRIVER = host_bin(os.path.join(ROOT, "tools", "lsp_scenarios"))

SCENARIOS = [f"Basic{i}" for i in range(1, 10)] + [f"SendReceive{i}" for i in range(1, 4)] + \
    [f"Robust{i}" for i in range(1, 7)] + [f"Window{i}" for i in range(1, 7)] + \
    ["ServerSlowStart1", "ServerSlowStart2", "ServerClose1", "ServerClose2", "ServerCloseConns1",
     "ServerCloseConns2", "ClientClose1", "ClientClose2"] + \
    [f"{m}{i}" for m in ("ServerFastClose", "ServerToClient", "ClientToServer", "RoundTrip") for i in range(1, 4)] + \
    ["VariableLengthMsgServer", "VariableLengthMsgClient"]
# not in the reference: Params::Copies > 1 (first transmissions sent k times)
# delivers every message exactly once, in order, with and without loss
DUPLICATE_SCENARIOS = ["DuplicatesExactlyOnce", "DuplicatesUnderDrop"]


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-s", "-C", ROOT, "tools/lsp_scenarios"], check=True)


def test_driver_lists_every_scenario():
    out = subprocess.run([DRIVER, "--list"], capture_output=True, text=True, check=True).stdout.split()
    assert sorted(out) == sorted(SCENARIOS + DUPLICATE_SCENARIOS)


@pytest.mark.parametrize("copies", [1, 2])
@pytest.mark.parametrize("name", SCENARIOS + DUPLICATE_SCENARIOS)
def test_reference_scenario(name, copies):
    """copies 1: the reference's protocol; copies 2: what the bitcoin
    programs run by default (lsp::DefaultAppCopies) -- the reference's
    scenarios must pass unchanged with every first transmission doubled."""
    if name in DUPLICATE_SCENARIOS and copies == 2:
        pytest.skip("sets its own Copies")
    r = subprocess.run([DRIVER, "--copies", str(copies), name], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith(f"{name} PASS")
