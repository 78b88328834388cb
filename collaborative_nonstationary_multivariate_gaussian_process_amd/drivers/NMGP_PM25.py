"""Drop-in for ``code/NMGP_PM25.py``: the PM2.5 driver ``VTVLCM`` (code/NMGP_PM25.py:53-117).

Length-scale logs fixed at 10 (``:63``), mu_v = 1 (``:64``).  Data: ``set_data`` / ``load_data`` /
``synthetic_data`` instead of the reference's import-time pickle load of ``../data/PM25/subdata.pickle``.
"""
import os

from . import _common

CFG = {"name": "PM25", "data_file": "subdata.pickle", "length_scale_log": 10, "show_elbo_without_test": True, "state": {}}


def set_data(X_list, Y_list, Xt_list, Yt_list):
    """Inject the four per-output lists the reference reads from its data pickle (:23-24)."""
    CFG["state"]["data"] = _common.DriverData(X_list, Y_list, Xt_list, Yt_list)


def load_data(path=None):
    """Read a data pickle in the reference layout (default: the reference's own relative path)."""
    CFG["state"]["data"] = _common.read_pickle(path or os.path.join("..", "data", CFG["name"], CFG["data_file"]))


def VTVLCM(data, M, batchsize=0, lr=0.01, itnum=2000, do_inference=True, do_test=False, res_dir="../res",
           **inference_kw):
    """code/NMGP_PM25.py:53-117.  Returns (model, loss_list, time_list), or with rmse_test_list when
    do_test.  Extra keyword arguments are passed to `inference` (device, noise, use_graph, dtype,
    show_ELBO, verbose, ...); res_dir=None skips the result pickle."""
    return _common.vtvlcm(CFG, data, M, batchsize, lr, itnum, do_inference, do_test, res_dir, dict(inference_kw))
