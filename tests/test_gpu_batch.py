"""GPU tests of the device-sharded batch handle (hs_batch_create / set_params / run /
hs_select_best, SURVEY.md 8b exports 2-5) through the C ABI.

On the one-GPU test box the mask holds device 0 only; the sharding arithmetic is the
one of hslabs_amd/dist.py (tests/test_dist.py), the per-device launches are hs_run's.
Bit-for-bit equality is expected against hs_run_host (same kernel, same inputs).
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hexapod(gpu):
    return gpu.KinematicModel(os.path.join(MODELS, "hexapod.xml"))


def test_batch_matches_run_host(gpu, hexapod):
    from hslabs_amd import synth

    params = synth.gen_params(1000, "hexapod")
    sb = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20)
    out = sb.run(k0=0, want=("q", "tau", "cf", "x", "flags", "work", "cot"))
    ref = gpu.run_host(hexapod, params, n_t=20, k0=0, horizon=20)
    for k in ("q", "tau", "cf", "x", "flags"):
        assert np.array_equal(out[k], ref[k]), k
    assert np.array_equal(out["work"], ref["work_cot"][:, 0])
    assert np.array_equal(out["cot"], ref["work_cot"][:, 1])


def test_select_best_is_min_key(gpu, hexapod):
    """hs_select_best = the lowest (float32 COT, id) key over the batch (measure_cot_sweep's
    minimum, ties to the lowest id)."""
    from hslabs_amd import capi, synth

    params = synth.gen_params(777, "hexapod")
    sb = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20)
    out = sb.run(k0=0)
    L = capi.load()
    sel = [L.hs_best_key_cot(float(w), hexapod.total_mass, float(l), 20, 20)
           for w, l in zip(out["work"], params["step_length"])]
    keys = [L.hs_best_key_encode(c, i) for i, c in enumerate(sel)]
    cot, rid = sb.select_best()
    kmin = min(keys)
    assert rid == kmin & 0xFFFFFFFF
    assert cot == np.float32(abs(out["cot"][rid]))


def test_select_best_over_a_one_rank_comm(gpu, hexapod):
    """hs_select_best_comm / hs_comm_reduce_best: the RCCL all-reduce(MIN) of the 8-byte key inside
    libhslabs, on a communicator of one rank (the one-GPU box); the N-rank layout is the launcher's
    (tests/test_bench_launcher.py)."""
    import torch

    from hslabs_amd import synth

    params = synth.gen_params(333, "hexapod")
    sb = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20)
    sb.run(k0=0)
    comm = gpu.Comm(1, 0, gpu.Comm.unique_id())
    local = sb.select_best()
    assert sb.select_best(comm) == local
    assert sb.select_best() == local  # the reduce ran in the comm's own buffer, not the batch's key
    key = torch.tensor([0x0123456789ABCDEF], dtype=torch.int64, device="cuda")
    comm.reduce_best(key)
    torch.cuda.synchronize()
    assert int(key.item()) == 0x0123456789ABCDEF
    # a rank whose batch has not run still completes the collective (contributing the largest key)
    # and then returns the error
    fresh = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20)
    with pytest.raises(gpu.capi.HSError):
        fresh.select_best(comm)
    assert sb.select_best(comm) == local  # the communicator is still usable
    comm.free()


def test_batch_run_into_device_buffers(gpu, hexapod):
    """hs_batch_run_device writes caller-owned device tensors; the same values as host outputs."""
    import torch

    from hslabs_amd import synth

    params = synth.gen_params(100, "hexapod")
    sb = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20)
    host = sb.run(k0=0, want=("tau", "cf", "flags", "work", "cot"))
    dev = {"tau": torch.zeros((100, 20, 18), dtype=torch.float64, device="cuda"),
           "cf": torch.zeros((100, 20, 18), dtype=torch.float64, device="cuda"),
           "flags": torch.zeros((100, 20), dtype=torch.int32, device="cuda"),
           "work": torch.zeros(100, dtype=torch.float64, device="cuda"),
           "cot": torch.zeros(100, dtype=torch.float64, device="cuda")}
    sb.run_device(dev, k0=0)
    for k, v in dev.items():
        got = v.cpu().numpy()
        assert np.array_equal(got.view(np.uint32) if k == "flags" else got, host[k]), k


def test_batch_run_device_rejects_bad_tensors(gpu, hexapod):
    """run_device checks every caller tensor before the native copy (which trusts the batch's sizes):
    wrong dtype, too small, non-contiguous, on the host or an unknown key all raise, and nothing
    is written."""
    import torch

    from hslabs_amd import synth

    sb = gpu.ShardedBatch(hexapod, synth.gen_params(16, "hexapod"), horizon=20, n_t=20)
    good = torch.zeros((16, 20, 18), dtype=torch.float64, device="cuda")
    bad = {"dtype": {"tau": good.float()},
           "shape": {"tau": good[:8]},
           "contiguous": {"tau": torch.zeros((16, 18, 20), dtype=torch.float64, device="cuda").transpose(1, 2)},
           "host": {"tau": good.cpu()},
           "key": {"torques": good},
           "flags dtype": {"flags": torch.zeros((16, 20), dtype=torch.float64, device="cuda")}}
    for what, out in bad.items():
        with pytest.raises(ValueError):
            sb.run_device(out, k0=0)
    assert not good.any().item(), "nothing may be written before the checks pass"
    sb.run_device({"tau": good}, k0=0)
    torch.cuda.synchronize()
    assert good.abs().sum().item() > 0


def test_batch_steps_and_fp32(gpu, hexapod):
    """H = 1 runs at successive k0 give the H = n_t rows; the fp32 batch follows the fp64 one."""
    from hslabs_amd import synth

    params = synth.gen_params(64, "hexapod")
    full = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20).run(k0=0)
    one = gpu.ShardedBatch(hexapod, params, horizon=1, n_t=20)
    for k0 in (0, 7, 19):
        o = one.run(k0=k0)
        assert np.array_equal(o["tau"][:, 0], full["tau"][:, k0])
    f32 = gpu.ShardedBatch(hexapod, params, horizon=20, n_t=20, fp32=True).run(k0=0)
    assert f32["tau"].dtype == np.float32
    same = (f32["flags"] == full["flags"]).all(axis=1)
    err = np.abs(f32["tau"][same] - full["tau"][same]) / np.maximum(1, np.abs(full["tau"][same]))
    assert same.mean() > 0.9 and err.max() < 1e-3


def test_batch_argument_errors(gpu, hexapod):
    import ctypes

    from hslabs_amd import capi

    L = capi.load()
    h = ctypes.c_void_p()
    assert L.hs_batch_create(hexapod.handle, 16, 1, 20, 0, 0, ctypes.byref(h)) != 0  # empty mask
    assert b"mask" in L.hs_last_error()
    assert L.hs_batch_create(hexapod.handle, 16, 1, 20, 0, 1 << 31, ctypes.byref(h)) != 0  # no such device
    assert L.hs_batch_create(hexapod.handle, 0, 1, 20, 0, 1, ctypes.byref(h)) != 0
    assert L.hs_batch_create(hexapod.handle, 16, 1, 20, 7, 1, ctypes.byref(h)) != 0  # precision
    assert L.hs_batch_create(hexapod.handle, 16, 1, 20, 0, 1, ctypes.byref(h)) == 0
    o = capi.BatchOutputsC()
    assert L.hs_batch_run(h, 0, 1, ctypes.byref(o)) != 0  # params not set
    c, i = ctypes.c_float(), ctypes.c_int64()
    assert L.hs_select_best(h, ctypes.byref(c), ctypes.byref(i)) != 0  # nothing run
    assert L.hs_batch_best_key_device(h, 0) is not None
    assert L.hs_batch_best_key_device(h, 1) is None
    L.hs_batch_free(h)
