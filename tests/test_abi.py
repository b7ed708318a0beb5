"""C-ABI boundary checks that need no GPU (include/trajmpc.h <-> libtrajmpc.so <-> ctypes).

- every function include/trajmpc.h declares is exported by the built library and bound in _lib._SIGS;
- the ctypes struct layouts equal the C compiler's (sizeof / offsetof from a gcc-compiled probe);
- host-only entry points (defaults, strings, workspace size, argument validation) behave as documented.
No compute entry point is launched here.
"""
import ctypes as C
import glob
import json
import os
import re
import subprocess

import numpy as np
import pytest

from trajectory_generation_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "trajmpc.h")
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))


def declared_functions():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(traj_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_every_declared_symbol_is_exported(L):
    names = declared_functions()
    assert len(names) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared in trajmpc.h but not exported: {missing}"
    unbound = [n for n in names if n not in _lib.exported_symbols()]
    assert not unbound, f"declared but not bound in _lib._SIGS: {unbound}"
    extra = [n for n in _lib.exported_symbols() if n not in names]
    assert not extra, f"bound in _lib but not declared: {extra}"


def _c_layout(tmp_path):
    structs = {"traj_vehicle_params": _lib.VehicleParams, "traj_mpc_config": _lib.MpcConfig,
               "traj_paths": _lib.Paths, "traj_knet_limits": _lib.KnetLimits}
    lines = ['#include <stdio.h>', '#include <stddef.h>'] + [f'#include "{h}"' for h in HEADERS] + ["int main(void) {",
             'printf("{");']
    first = True
    for sname, cls in structs.items():
        items = [f'\\"sizeof\\": %zu'] + [f'\\"{f}\\": %zu' for f, _ in cls._fields_]
        args = [f"sizeof({sname})"] + [f"offsetof({sname}, {f})" for f, _ in cls._fields_]
        sep = "" if first else ","
        first = False
        lines.append(f'printf("{sep}\\"{sname}\\": {{{", ".join(items)}}}", {", ".join(args)});')
    lines += ['printf("}\\n");', "return 0; }"]
    c_file = tmp_path / "layout.c"
    c_file.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(c_file)], check=True)
    return json.loads(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout), structs


def test_struct_layout_matches_c(tmp_path):
    layout, structs = _c_layout(tmp_path)
    for sname, cls in structs.items():
        got = layout[sname]
        assert got["sizeof"] == C.sizeof(cls), sname
        for f, _ in cls._fields_:
            assert got[f] == getattr(cls, f).offset, f"{sname}.{f}"


def test_abi_version_and_strings(L):
    assert L.traj_abi_version() == 4
    for code, s in _lib.STATUS_STRINGS.items():
        assert L.traj_status_string(code).decode() == s
    for rc in (_lib.TRAJ_OK, _lib.TRAJ_E_ARG, _lib.TRAJ_E_UNSUPPORTED, _lib.TRAJ_E_LAUNCH):
        assert L.traj_error_string(rc)


def test_default_params_are_the_reference_params(L):
    from trajectory_generation_amd.batch import REFERENCE_PARAMS
    p = _lib.default_params()
    for k, v in REFERENCE_PARAMS.items():
        assert getattr(p, k) == v, k


def test_default_config_matches_oracle(L, oracle_lib):
    O = oracle_lib
    for N, Ts in ((20, 0.02), (40, 0.05), (1, 0.1)):
        c = _lib.default_config(N, Ts)
        o = O.cfg(N=N, Ts=Ts)
        for f, _ in _lib.MpcConfig._fields_:
            if f == "warm_start":      # closed-loop option of the HIP path, off in the oracle by default
                continue
            a, b = getattr(c, f), getattr(o, f)
            if isinstance(a, (int, float)):
                assert a == b, f
            else:
                assert list(a) == list(b), f
        # mpc_6stati.py:120-143 defaults
        assert (c.q_c, c.q_phi, c.q_vx) == (6.0, 0.5, 0.5)
        assert list(c.R) == [0.02, 0.0, 0.0, 2.0] and list(c.Rd) == [0.01, 0.0, 0.0, 5.0]
        assert list(c.u_lo) == [-1.0, -0.6] and list(c.u_hi) == [1.0, 0.6]
        assert list(c.du_lo) == [-0.5, -0.3] and list(c.du_hi) == [0.5, 0.3]
        assert (c.eps_abs, c.eps_rel, c.max_iter, c.polish) == (1e-5, 1e-5, 10000, 1)


def test_workspace_bytes(L):
    """The base part (A/B/g, stage records, warm records, order, queue) and, for the row-split kernel's horizons
    (TRAJ_SPLIT_MIN_N <= N <= TRAJ_MAX_N_SPLIT, mpc_split.h), its P scratch: NRW x 2H doubles per instance + 16 bytes
    of alignment slack (H = 40 / 48 / 64 by n = 2N; NRW = 32 rows per wave)."""
    def split(B, N):
        if not (_lib.SPLIT_MIN_N <= N <= _lib.MAX_N_SPLIT):
            return 0
        H = 40 if 2 * N <= 80 else (48 if 2 * N <= 96 else 64)
        return (B * 32 * ((2 * H + 31) // 32) * 2 * H + 2) * 8
    for B, N in ((0, 20), (1, 1), (4096, 20), (7, 40), (7, 21), (3, 48), (2, 64), (2, 65)):
        assert L.traj_mpc_workspace_bytes(B, N) == ((B * N * 66 + 4 * B) * 8 + ((4 * (3 * B + 2) + 7) // 8) * 8
                                                    + split(B, N)), (B, N)
    assert L.traj_mpc_workspace_bytes(-1, 20) == 0


def test_state_bound_workspace_bytes(L):
    """The state-bound solver's scratch is caller-owned (mpc_general.h gen_ws_doubles per instance)."""
    def per(N):
        n, m = 2 * N, 10 * N
        return (n * n + m * n + 6 * (N + 1) * n + 6 * (N + 1) + 3 * n + 20 * n + 24 * m + 64 +
                (n * n if N > _lib.MAX_N else 0))   # past the hot capacity the Cholesky factor leaves LDS
    for B, N in ((0, 20), (1, 1), (4096, 20), (7, 40), (3, 41), (2, 60), (1, _lib.MAX_N_GENERAL)):
        assert L.traj_mpc_sb_workspace_bytes(B, N) == B * per(N) * 8
    assert L.traj_mpc_sb_workspace_bytes(-1, 20) == 0
    assert L.traj_mpc_sb_workspace_bytes(4, _lib.MAX_N_GENERAL + 1) == 0


def test_long_horizon_scratch_fits_the_state_bound_region():
    """The long-horizon kernel (mpc_long.h, TRAJ_MAX_N < N <= TRAJ_MAX_N_LONG) takes its scratch from the same
    caller-owned region: the scaled P, ld x ld column-major with ld = n rounded up to 8, and K^-1 beside it past
    n = 128 (below, K^-1 is in LDS) -- never more than traj_mpc_sb_workspace_bytes gives per instance."""
    def gen(N):
        n, m = 2 * N, 10 * N
        return n * n + m * n + 6 * (N + 1) * n + 6 * (N + 1) + 3 * n + 20 * n + 24 * m + 64 + n * n
    for N in range(_lib.MAX_N + 1, _lib.MAX_N_LONG + 1):
        n = 2 * N
        ld = (n + 7) // 8 * 8
        assert ld * ld * (2 if n > 128 else 1) <= gen(N), N
    assert _lib.MAX_N < _lib.MAX_N_LONG <= _lib.MAX_N_GENERAL


def test_argument_errors_are_reported_before_any_launch(L):
    p = _lib.default_params()
    c = _lib.default_config(20, 0.05)
    nul = None
    # null params / negative batch
    assert L.traj_mpc_step_batch(None, C.byref(c), 4, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_E_ARG
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(c), -1, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_E_ARG
    # empty batch is a no-op
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(c), 0, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_OK
    # horizon beyond the general solver's capacity / non-positive horizon
    for N in (0, _lib.MAX_N_GENERAL + 1):
        cN = _lib.default_config(20, 0.05)
        cN.N = N
        assert L.traj_mpc_step_batch(C.byref(p), C.byref(cN), 0, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_E_ARG
    # past the hot kernels' capacity: the step / QP entry points take it (the row-split kernel up to TRAJ_MAX_N_SPLIT,
    # its scratch inside traj_mpc_workspace_bytes; past it the long-horizon / general solvers, their scratch after it:
    # a workspace without it is refused before launching)
    cL = _lib.default_config(60, 0.05)
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(cL), 0, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_OK
    fk = C.c_void_p(16)
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(cL), 4, *([fk] * 11), fk,
                                 L.traj_mpc_workspace_bytes(4, 60) - 8, nul) == _lib.TRAJ_E_ARG
    cLL = _lib.default_config(_lib.MAX_N_SPLIT + 1, 0.05)
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(cLL), 4, *([fk] * 11), fk,
                                 L.traj_mpc_workspace_bytes(4, _lib.MAX_N_SPLIT + 1), nul) == _lib.TRAJ_E_ARG
    assert L.traj_mpc_qp_batch(C.byref(p), C.byref(cL), 4, *([fk] * 14), nul, 0, nul) == _lib.TRAJ_E_ARG
    assert L.traj_closed_loop_check(nul, 0, 4, 60, nul) == _lib.TRAJ_E_ARG
    # workspace too small (checked before launching)
    fake = C.c_void_p(16)
    args = [fake] * 11
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(c), 4, *args, fake, 8, nul) == _lib.TRAJ_E_ARG
    # state bounds run on the general solver for the step / QP entry points; the closed loop (whose
    # reference caller never passes them) reports them as unsupported, never silently ignored
    cx = _lib.default_config(20, 0.05)
    cx.has_x_lo = 1
    for i in range(6):
        cx.x_lo[i] = -1e3
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(cx), 0, *([nul] * 11), nul, 0, nul) == _lib.TRAJ_OK
    # ... with caller-owned scratch: a workspace without the state-bound part is refused before launching
    base = L.traj_mpc_workspace_bytes(4, 20)
    assert L.traj_mpc_step_batch(C.byref(p), C.byref(cx), 4, *args, fake, base, nul) == _lib.TRAJ_E_ARG
    assert L.traj_mpc_qp_batch(C.byref(p), C.byref(cx), 4, *([fake] * 14), nul, 0, nul) == _lib.TRAJ_E_ARG
    assert L.traj_mpc_qp_batch(C.byref(p), C.byref(cx), 4, *([fake] * 14), fake,
                               L.traj_mpc_sb_workspace_bytes(4, 20) - 8, nul) == _lib.TRAJ_E_ARG
    ps = _lib.Paths()
    ps.kmax, ps.kind, ps.pc = 0, 16, 16                      # never dereferenced at B = 0
    # the closed loop takes them too (ABI 4: one step per launch sequence on the general solver), with its scratch
    # (traj_closed_loop_workspace_bytes: the general solver's plus the step's window and u_cmd) -- a workspace without
    # it is an argument error before any launch
    assert L.traj_closed_loop_step(C.byref(p), C.byref(cx), C.byref(ps), 0, nul, nul, nul, 0, 0, nul, nul, nul,
                                   nul, nul, 0, nul) == _lib.TRAJ_OK
    wcx = L.traj_closed_loop_workspace_bytes(C.byref(cx), 4)
    assert wcx >= base + L.traj_mpc_sb_workspace_bytes(4, 20) + 4 * (3 * 21 + 2) * 8
    assert L.traj_closed_loop_workspace_bytes(C.byref(c), 4) == base
    assert L.traj_closed_loop_step(C.byref(p), C.byref(cx), C.byref(ps), 4, fake, fake, fake, 0, 0, nul, nul, nul,
                                   nul, fake, wcx - 8, nul) == _lib.TRAJ_E_ARG
    assert L.traj_closed_loop_run(C.byref(p), C.byref(cx), C.byref(ps), 4, fake, fake, fake, 0, 1, 0, nul, nul, nul,
                                  nul, fake, wcx - 8, nul) == _lib.TRAJ_E_ARG
    # horizons past the hot kernels' capacity: the closed loop takes them up to TRAJ_MAX_N_LONG (past TRAJ_MAX_N_SPLIT
    # the long-horizon kernel, whose scratch follows the workspace -- a workspace without it is an argument error
    # before any launch); past that, and with state bounds, the general solver up to TRAJ_MAX_N_GENERAL (the step's own
    # limit; past it an argument error, as for the step)
    cL = _lib.default_config(_lib.MAX_N_SPLIT + 4, 0.05)
    cG = _lib.default_config(_lib.MAX_N_LONG + 1, 0.05)
    cLx = _lib.default_config(_lib.MAX_N_GENERAL + 1, 0.05)
    cLx.has_x_lo, cLx.x_lo[3] = 1, -1.0
    assert L.traj_closed_loop_workspace_bytes(C.byref(cLx), 4) == 0
    assert L.traj_closed_loop_workspace_bytes(C.byref(cG), 4) > L.traj_mpc_sb_workspace_bytes(4, _lib.MAX_N_LONG + 1)
    wsL = L.traj_mpc_workspace_bytes(4, _lib.MAX_N_SPLIT + 4)
    for fn in (L.traj_closed_loop_step, L.traj_closed_loop_run):
        extra = (0, 1) if fn is L.traj_closed_loop_run else (0,)
        assert fn(C.byref(p), C.byref(cL), C.byref(ps), 0, nul, nul, nul, *extra, 0, nul, nul, nul, nul, nul, 0,
                  nul) == _lib.TRAJ_OK
        assert fn(C.byref(p), C.byref(cL), C.byref(ps), 4, fake, fake, fake, *extra, 0, nul, nul, nul, nul, fake, wsL,
                  nul) == _lib.TRAJ_E_ARG
        assert fn(C.byref(p), C.byref(cG), C.byref(ps), 0, nul, nul, nul, *extra, 0, nul, nul, nul, nul, nul, 0,
                  nul) == _lib.TRAJ_OK
        assert fn(C.byref(p), C.byref(cLx), C.byref(ps), 0, nul, nul, nul, *extra, 0, nul, nul, nul, nul, nul, 0,
                  nul) == _lib.TRAJ_E_ARG


def test_check_raises():
    with pytest.raises(RuntimeError):
        _lib.check(_lib.TRAJ_E_ARG, "x")
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.TRAJ_E_UNSUPPORTED, "x")
    _lib.check(_lib.TRAJ_OK, "x")


def test_product_path_has_no_oracle_dependency():
    """The shipped package must not import, call or link anything under oracle/."""
    pkg = os.path.join(ROOT, "trajectory_generation_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")) or f == "Makefile":
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle\b|traj_oracle|pyoracle", src, flags=re.M), f
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "traj_oracle" not in out


def test_bench_spawns_one_worker_per_gpu(monkeypatch):
    """`bench.py --gpus N` without a launcher starts N worker processes (RANK / LOCAL_RANK / WORLD_SIZE,
    rendezvous on 127.0.0.1) from a parent that never touches the GPU, and fails when a worker fails."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    started = []

    class P:
        def __init__(self, cmd, env):
            started.append((cmd, env))

        def poll(self):
            return 0

        def wait(self, timeout=None):
            return 0

    monkeypatch.setattr(subprocess, "Popen", P)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    bench._spawn_workers(4)
    assert [e["RANK"] for _, e in started] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["LOCAL_RANK"] == e["RANK"] and e["MASTER_ADDR"] == "127.0.0.1"
               for _, e in started)
    assert all(c[-4:] == ["--gpus", "4", "--steps", "3"] and c[1].endswith("bench.py") for c, _ in started)
    assert "torch.cuda" not in sys.modules or not __import__("torch").cuda.is_initialized()
