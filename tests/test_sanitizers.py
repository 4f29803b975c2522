"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

Two builds, no GPU:
  * csrc/sanitize.mk: the C ABI's host half (zb_host.cpp: model / config validation, the team
    topology zb_create uploads, the defaults) with a mutation driver that feeds check_model tens of
    thousands of corrupted models; a corrupted index that validation lets through and the topology
    builder then follows out of its array aborts the run.
  * oracle/asan.mk: the CPU twin (zb_oracle.c) stepping envs with pushes, randomization, automatic
    and masked resets through every output.
"""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")
ORACLE = os.path.join(ROOT, "oracle")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _blobs(tmp_path, cm, **cfg_kw):
    from zbot_amd import default_config

    m, c = tmp_path / "model.bin", tmp_path / "config.bin"
    m.write_bytes(bytes(cm.cmodel))
    c.write_bytes(bytes(default_config(solver="newton", **cfg_kw)))
    return str(m), str(c)


def _run(cmd, timeout):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0, f"{cmd[0]} rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_host_validation_under_sanitizers(tmp_path, cmodel):
    subprocess.run(["make", "-C", CSRC, "-s", "-f", "sanitize.mk"], check=True)
    m, c = _blobs(tmp_path, cmodel)
    out = _run([os.path.join(CSRC, "build", "zb_host_selftest"), m, c, "30000"], timeout=300)
    assert "zb_host_selftest ok: 30000 mutations" in out
    rejected = int(out.split("accepted, ")[1].split(" rejected")[0])
    assert rejected > 3000  # the corruptions do reach the checks


def test_host_validation_rejects_bad_indices(tmp_path, cmodel):
    """The index checks the sanitizer run found necessary, through the product library's zb_create
    (returns before touching a device)."""
    import ctypes as C

    from zbot_amd import default_config
    from zbot_amd import engine as E

    L = E.load_library()
    cases = [("dof_parent", 20, 999), ("geom_body", 0, 40), ("site_imu", None, 7), ("act_dof", 3, -2),
             ("body_parent", 5, 9), ("level_nmem", 0, 12), ("dof_rowoff", 7, 5000)]
    for field, idx, val in cases:
        bad = type(cmodel.cmodel).from_buffer_copy(cmodel.cmodel)
        if idx is None:
            setattr(bad, field, val)
        else:
            getattr(bad, field)[idx] = val
        h = C.c_void_p()
        rc = L.zb_create(C.byref(bad), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
        assert rc == -4, (field, rc, L.zb_last_error())


@pytest.mark.slow
def test_oracle_twin_under_sanitizers(tmp_path, cmodel):
    subprocess.run(["make", "-C", ORACLE, "-s", "-f", "asan.mk"], check=True)
    m, c = _blobs(tmp_path, cmodel, push=True, randomize=True, max_episode_sec=0.5)
    out = _run([os.path.join(ORACLE, "_asan", "zb_oracle_selftest"), m, c, "16", "40"], timeout=600)
    assert "zb_oracle_selftest ok" in out and "episode ends 0" not in out
