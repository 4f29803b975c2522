"""The counting build of the CPU twin (oracle/zb_flops.cpp, SURVEY §8(d) FLOP count) computes the
same states as the plain fp32 twin, bit for bit, and counts arithmetic."""
import ctypes as C

import numpy as np


def test_counting_twin_is_the_twin(cmodel, oracle_mod):
    from zbot_amd import default_config

    O = oracle_mod
    cfg = default_config(solver="newton")
    n, seed = 4, 5
    a = O.OracleEnv(cmodel.cmodel, cfg, n, seed=seed)
    b = O.OracleEnv(cmodel.cmodel, cfg, n, seed=seed, precision="flops")
    a.reset()
    b.reset()
    L = O.lib("flops")
    L.zbo_flops_reset()
    for t in range(6):
        act = O.synthetic_actions(cmodel.cmodel, seed, n, 0, t)
        ra, rb = a.step(act), b.step(act)
        for k in ra:
            np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
        np.testing.assert_array_equal(a.state, b.state)
        np.testing.assert_array_equal(a.iters, b.iters)
    out = (C.c_uint64 * 6)()
    L.zbo_flops_get(out)
    add, mul, div, sqrt, trans, cmp = out
    assert add > 0 and mul > 0 and div > 0 and sqrt > 0 and trans > 0 and cmp > 0
    per_step = (add + mul + div + sqrt + trans) / (n * 6)
    assert 1e5 < per_step < 1e8
