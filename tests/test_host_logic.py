"""Host-side logic that needs no GPU: the on-device pipeline's index loader draws the reference
DataLoader's batches, the drivers keep the reference signatures, the re-saved model.pt fixture equals
the shipped checkpoint, and the data-parallel batch split / skip rule is consistent over ranks."""
import inspect
import os

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader

from collaborative_nonstationary_multivariate_gaussian_process_amd import distributed as DD
from collaborative_nonstationary_multivariate_gaussian_process_amd import nmgp_dsvi as NM

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_MODEL_PT = "/root/reference/code/notebook/model.pt"


@pytest.mark.parametrize("N,bs", [(200, 200), (10000, 2000), (1003, 128), (37, 5)])
def test_index_loader_draws_the_reference_batches(N, bs):
    """Same global-RNG draws and the same row order as DataLoader(trainData(X, Y, I), shuffle=True)
    (code/nmgp_dsvi.py:816-817): the device pipeline gathers exactly the reference's minibatches."""
    X = torch.arange(N, dtype=torch.float64) * 0.5
    Y = -X
    I = (torch.arange(N) % 3).to(torch.float64)
    torch.manual_seed(123)
    ref = [xb.clone() for xb, _, _ in DataLoader(NM.trainData(X, Y, I), batch_size=bs, shuffle=True)]
    after_ref = torch.randn(3)
    torch.manual_seed(123)
    got = [X[idx] for idx in NM._index_loader(N, bs)]
    after_got = torch.randn(3)
    assert len(ref) == len(got)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    assert torch.equal(after_ref, after_got)          # the generator advanced identically


def test_index_loader_with_private_generator_is_rank_independent():
    g1, g2 = torch.Generator().manual_seed(7), torch.Generator().manual_seed(7)
    torch.manual_seed(1)
    a = [b.clone() for b in NM._index_loader(500, 64, g1)]
    torch.randn(1000)                                   # other consumers of the global stream
    b = [b.clone() for b in NM._index_loader(500, 64, g2)]
    assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_vec2list_order_equals_stable_sort_by_output():
    """The device pipeline groups a minibatch by a stable sort on the output id: vec2list's order."""
    rng = np.random.default_rng(0)
    I = torch.from_numpy(rng.integers(0, 5, 300).astype(np.float64))
    X = torch.from_numpy(rng.uniform(size=300))
    xl, _ = NM.vec2list(X, X, I, dim=5)
    order = torch.sort(I.long(), stable=True).indices
    assert torch.equal(torch.cat(xl), X[order])


@pytest.mark.parametrize("n,world", [(7, 2), (8, 3), (2001, 8), (1, 2)])
def test_rank_slices_cover_each_row_once(n, world):
    rows = []
    for r in range(world):
        s, e = DD.shard_bounds(n, r, world)
        rows += list(range(s, e))
    assert rows == list(range(n))
    sizes = [DD.shard_bounds(n, r, world)[1] - DD.shard_bounds(n, r, world)[0] for r in range(world)]
    assert max(sizes) - min(sizes) <= 1
    # the inference loop skips a global batch with fewer rows than ranks on EVERY rank
    assert (n < world) == (min(sizes) == 0)


def test_drivers_keep_reference_signatures():
    from collaborative_nonstationary_multivariate_gaussian_process_amd.drivers import NMGP_HCP, NMGP_PM25
    for mod, ls in ((NMGP_PM25, 10), (NMGP_HCP, 5)):
        sig = inspect.signature(mod.VTVLCM)
        params = list(sig.parameters.values())
        # code/NMGP_PM25.py:53 / code/NMGP_HCP.py:51
        assert [p.name for p in params[:7]] == ["data", "M", "batchsize", "lr", "itnum", "do_inference", "do_test"]
        assert [params[i].default for i in range(2, 7)] == [0, 0.01, 2000, True, False]
        assert mod.CFG["length_scale_log"] == ls
    with pytest.raises(RuntimeError, match="no PM25 data"):
        NMGP_PM25.CFG["state"].pop("data", None)
        NMGP_PM25.VTVLCM("PM25", 8, do_inference=True, res_dir=None)


def test_inference_signature_extends_the_reference():
    sig = inspect.signature(NM.inference)
    names = list(sig.parameters)
    ref = ["X_train_list", "Y_train_list", "z", "batch_size", "dim_outputs", "hyperpars", "fix_hyperpars", "mu_v",
           "mu_W", "mu_U", "sqrt_v", "sqrt_W", "sqrt_U", "lr", "itnum", "do_stop_criterion", "seed", "verbose", "PATH",
           "continuous_training", "show_ELBO", "save_model", "X_test_list", "Y_test_list"]   # code/nmgp_dsvi.py:758-761
    assert names[:len(ref)] == ref


def test_modelpt_fixture_matches_the_shipped_checkpoint():
    fx = torch.load(os.path.join(ROOT, "tests", "golden", "model_pt.pt"), weights_only=True)
    assert fx["epoch"] == 1999 and float(fx["loss"]) == pytest.approx(151.0889, abs=1e-3)
    assert list(fx["model_state_dict"].keys())[0] == "mu_W" and len(fx["model_state_dict"]) == 13
    if not os.path.exists(REF_MODEL_PT):
        pytest.skip("reference tree not present (GPU box); fixture checked in the build container")
    ck = torch.load(REF_MODEL_PT, weights_only=True, map_location="cpu")
    for k, v in ck["model_state_dict"].items():
        assert torch.equal(v, fx["model_state_dict"][k]), k
    so, sf = ck["optimizer_state_dict"], fx["optimizer_state_dict"]
    assert so["param_groups"][0]["params"] == sf["param_groups"][0]["params"]
    for pid, st in so["state"].items():
        assert torch.equal(st["exp_avg"], sf["state"][pid]["exp_avg"])
        assert torch.equal(st["exp_avg_sq"], sf["state"][pid]["exp_avg_sq"])
        assert int(st["step"]) == int(float(sf["state"][pid]["step"]))


# ------------------------------------------------------------------------------ driver data loader
@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_driver_data_pickle_loader_reads_numpy_lists(tmp_path, protocol):
    """drivers._dataload reads the reference drivers' data layout ([X_list, Y_list, Xt_list, Yt_list] of
    numpy arrays, code/NMGP_PM25.py:26-28) from pickles of every protocol without unpickling them."""
    import pickle
    from collaborative_nonstationary_multivariate_gaussian_process_amd.drivers._dataload import load_data_pickle
    rng = np.random.default_rng(protocol)
    obj = [[rng.standard_normal((7, 1)), rng.standard_normal((5, 1)).astype(np.float32)],
           [np.arange(6, dtype=np.int64).reshape(3, 2), np.asfortranarray(rng.standard_normal((3, 4)))],
           [rng.standard_normal(0)], [np.array(2.5)], {"t_max": 1.5, "name": "pm25", "b": b"xy"}, (1, None, True)]
    p = tmp_path / "d.pickle"
    p.write_bytes(pickle.dumps(obj, protocol=protocol))
    got = load_data_pickle(str(p))
    for a, b in zip(got[:4], obj[:4]):
        for x, y in zip(a, b):
            assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y)
    assert got[4] == obj[4] and tuple(got[5]) == obj[5]


class _Evil:
    def __reduce__(self):
        import os
        return (os.system, ("echo pwned > /dev/null",))


def test_driver_data_pickle_loader_refuses_code(tmp_path):
    import pickle
    from collaborative_nonstationary_multivariate_gaussian_process_amd.drivers._dataload import load_data_pickle
    for bad in ([np.zeros(3), _Evil()], [np.array([object()], dtype=object)]):
        p = tmp_path / "bad.pickle"
        p.write_bytes(pickle.dumps(bad, protocol=3))
        with pytest.raises(ValueError):
            load_data_pickle(str(p))


def test_driver_data_pickle_loader_reads_reference_toy_pickle():
    """The reference's shipped simulation pickle (build container only: skipped where the tree is absent)."""
    import os
    path = "/root/reference/data/simulation/sim_illustration_low_freq.pickle"
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    from collaborative_nonstationary_multivariate_gaussian_process_amd.drivers._dataload import load_data_pickle
    obj = load_data_pickle(path)
    assert len(obj) == 4 and all(len(l) == 2 for l in obj)
    arrs = [a for l in obj for a in l]
    assert all(isinstance(a, np.ndarray) and a.dtype == np.float64 and a.shape == (100, 1) for a in arrs)
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "toy_forward.npz"))
    assert np.array_equal(np.concatenate([a.reshape(-1) for a in obj[0]]), g["x"])
    assert np.array_equal(np.concatenate([a.reshape(-1) for a in obj[1]]), g["y"])


def test_split_k_rules():
    """GemmGroup's split-K choices (hip_ops): the automatic rule splits only tiny groups and problems far
    beyond the balanced per-workgroup share; the k-tile cap (kt_cap, round 3: 20 for the fp64 P-bar_G
    group) only raises a split, to at most 16 chunks.  PM2.5 P-bar_G: output D-1 runs k = 5 x 256 = 40 k-tiles
    -> 2 chunks, output 0 (8 k-tiles) stays whole."""
    from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H
    assert H._auto_ksplit(1280, 640, 5) == 1                 # PM2.5 P-bar_G under the automatic rule
    assert H._cap_ksplit(1, 1280, 20) == 2 and H._cap_ksplit(1, 256, 20) == 1
    assert H._cap_ksplit(1, 1024, 20) == 2 and H._cap_ksplit(1, 768, 20) == 2
    assert H._cap_ksplit(3, 256, 20) == 3                    # never lowered
    assert H._cap_ksplit(1, 10 ** 6, 2) == 16                # at most 16 chunks
    assert H._cap_ksplit(5, 10 ** 6, 0) == 5                 # 0: no cap
    assert H._auto_ksplit(2000, 16, 100) > 1                 # tiny groups split long k loops


def test_bench_refuses_gpus_world_mismatch():
    """bench.py --gpus N under a launcher whose WORLD_SIZE differs exits non-zero before touching the GPU
    (it never reports n_gpus != N); without a launcher N > 1 re-runs under torchrun (checked on the box)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_adam_lower_gate_needs_vector_aligned_blocks():
    """the triangular Adam only where M and every sqrt block offset are multiples of 16 / element size;
    round 6: from M = 256 on (one launch over the flat vector), toy shapes below keep the dense update."""
    import torch
    from collaborative_nonstationary_multivariate_gaussian_process_amd.engine import param_layout, use_adam_lower
    for D, M, dt, want in [(2, 512, torch.float32, True), (2, 514, torch.float32, False),
                           (2, 513, torch.float64, False), (2, 1024, torch.float64, True),
                           (2, 256, torch.float32, True), (5, 256, torch.float64, True), (2, 250, torch.float64, False),
                           (2, 20, torch.float64, False)]:
        offs, _ = param_layout(D, M)
        assert use_adam_lower(M, dt, offs) is want, (D, M, dt)
