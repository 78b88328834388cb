"""Shared body of the two VTVLCM drivers (code/NMGP_PM25.py:53-117, code/NMGP_HCP.py:51-118)."""
import os
import pickle

import numpy as np

from ._dataload import load_data_pickle


class DriverData:
    """The module-level arrays the reference drivers derive from their data pickle
    (code/NMGP_PM25.py:26-40): per-output train / test lists as (n, 1) columns, t_max."""

    def __init__(self, X_list, Y_list, Xt_list, Yt_list):
        col = lambda a: np.asarray(a, np.float64).reshape(-1)[:, None]
        self.X_list = [np.asarray(x, np.float64).reshape(-1) for x in X_list]
        self.Xt_list = [np.asarray(x, np.float64).reshape(-1) for x in Xt_list]
        self.X_train_list = [col(x) for x in X_list]
        self.X_test_list = [col(x) for x in Xt_list]
        self.Y_train_list = [col(y) for y in Y_list]
        self.Y_test_list = [col(y) for y in Yt_list]
        self.X_train_vec = np.concatenate(self.X_train_list)
        self.t_max = float(np.max([np.max(np.concatenate(self.X_list)), np.max(np.concatenate(self.Xt_list))]))
        self.n_dims = len(self.X_list)


def read_pickle(path):
    """A data file in the reference layout: pickle of [X_list, Y_list, Xt_list, Yt_list] (numpy arrays),
    read with the data-only loader (_dataload: the pickle is interpreted, never unpickled; anything but
    numpy array data is refused).  Only for files the user supplies; the reference ships none."""
    X_list, Y_list, Xt_list, Yt_list = load_data_pickle(path)
    return DriverData(X_list, Y_list, Xt_list, Yt_list)


def synthetic_data(n_outputs, n_train, n_test=0, t_max=1.0, seed=0):
    """Seeded synthetic series of the drivers' shape: per output, sorted inputs on
    [0, t_max] and smooth, output-correlated responses plus noise."""
    rng = np.random.default_rng(seed)
    X, Y, Xt, Yt = [], [], [], []
    base = rng.standard_normal(3)
    for d in range(n_outputs):
        x = np.sort(rng.uniform(0, t_max, n_train + n_test))
        f = np.sin(2 * np.pi * x / t_max * (1 + 0.2 * d) + base[0]) + 0.3 * np.cos(5 * np.pi * x / t_max + base[1] * d)
        y = f + 0.2 * rng.standard_normal(x.shape)
        test = np.zeros(x.shape, bool)
        if n_test:
            test[rng.choice(x.size, n_test, replace=False)] = True
        X.append(x[~test]); Y.append(y[~test]); Xt.append(x[test] if n_test else x[:1]); Yt.append(y[test] if n_test else y[:1])
    return X, Y, Xt, Yt


def vtvlcm(cfg, data, M, batchsize, lr, itnum, do_inference, do_test, res_dir, inference_kw):
    """The common VTVLCM body: z = linspace(0, t_max, M), fixed length-scale hyper-parameters,
    mu_v = 1, `inference`, result pickle ``{res_dir}/{data}/prediction_res_M{M}_B{batchsize}.pickle``."""
    from ..nmgp_dsvi import inference
    dd = cfg["state"].get("data")
    if dd is None:
        raise RuntimeError(f"no {cfg['name']} data: call set_data(X_list, Y_list, Xt_list, Yt_list), "
                           "load_data(path) or set_data(*synthetic_data(...)) first")
    z = np.linspace(0, dd.t_max, num=M)
    dim_outputs = len(dd.X_list)
    batch_size = dd.X_train_vec.shape[0] if batchsize == 0 else batchsize
    path = None if res_dir is None else os.path.join(res_dir, data, "prediction_res_M{}_B{}.pickle".format(M, batchsize))
    if do_inference:
        ls = cfg["length_scale_log"]
        hyperpars = {"length_scales_L0_log": ls, "length_scales_L1_log": ls, "length_scales_tildeell_log": ls}
        initpars = {"mu_v": 1 * np.ones(M)}
        kw = dict(lr=lr, itnum=itnum, hyperpars=hyperpars, verbose=inference_kw.pop("verbose", True))
        kw.update(initpars)
        kw.update(inference_kw)
        if do_test:
            out = inference(dd.X_train_list, dd.Y_train_list, z, batch_size, dim_outputs,
                            show_ELBO=kw.pop("show_ELBO", False), X_test_list=dd.X_test_list,
                            Y_test_list=dd.Y_test_list, **kw)
        else:
            # (the reference PM2.5 driver passes the test lists here too and then unpacks three of the
            # four returned values, code/NMGP_PM25.py:73-75 -- a ValueError; this driver does not pass them)
            kw.setdefault("show_ELBO", cfg["show_elbo_without_test"])
            out = inference(dd.X_train_list, dd.Y_train_list, z, batch_size, dim_outputs, **kw)
        if res_dir is not None:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "wb") as res:
                pickle.dump(list(out), res)
        return tuple(out)
    if path is None:
        raise ValueError("do_inference=False reloads an earlier run's result pickle: res_dir must be given")
    # do_inference=False: reload the results of an earlier run OF THIS DRIVER (it wrote the file above: whole
    # NMGP objects and lists, as the reference's result pickles, code/NMGP_PM25.py:101-113) -- the driver's
    # own output, not a user data file; user data goes through read_pickle's data-only loader
    with open(path, "rb") as res:
        return tuple(pickle.load(res))
