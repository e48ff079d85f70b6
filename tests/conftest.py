"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` tests run on any CPU box (oracle vs golden fixtures, host logic, the C ABI's
symbol table). `-m gpu` tests need a MI355X and call the HIP library through the C ABI."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "video-blade_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


# name -> list of facts recorded by tests and printed in the terminal summary (e.g. how many of the
# reference-golden cases reproduced the reference's mask bit for bit)
RECORD = {}


def record(name, fact):
    RECORD.setdefault(name, []).append(fact)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and libvblade_hip.so")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    for name, facts in RECORD.items():
        terminalreporter.write_line(f"[vblade record] {name}: {facts}")
