"""Drop-in API, host side (no GPU): module surface, reference-identical model
init and user partitions (RNG call order), plugin-by-name, no CPU path."""
import numpy as np
import pytest
import torch

from conftest import golden, load_project


def test_weighted_average_surface():
    m = load_project("weighted_average", ["simulators", "clients", "utils", "models", "sampling"])
    for name in ("Simulator", "NoConsDecFedAvg", "DecFedAvg", "Centeralized", "FedLCon", "GossipLearning"):
        assert hasattr(m["simulators"], name)
    for meth in ("communication_graph", "Neighbors", "run", "report", "select_global_model"):
        assert hasattr(m["simulators"].Simulator, meth)
    for meth in ("local_update", "consensus", "inference", "train_val_test", "report"):
        assert hasattr(m["clients"].Client, meth)
    for f in ("DotDict", "setup_seed", "DatasetSplit", "get_dataset", "exp_details", "servers_plot"):
        assert hasattr(m["utils"], f)


def test_primal_dual_surface():
    m = load_project("primal_dual", ["servers", "clients", "utils", "models", "sampling"])
    for name in ("Server", "FedAvg_Server", "FedProx_Server", "FedAdmm_Server"):
        assert hasattr(m["servers"], name)
    for meth in ("average_weights", "run", "avg_trainig_calculator", "update_global_model", "tarining", "plot"):
        assert hasattr(m["servers"].FedAdmm_Server, meth)
    m2 = load_project("primal_dual", ["utils"])
    for f in ("DotDict", "setup_seed", "DatasetSplit", "get_dataset", "exp_details", "servers_plot"):
        assert hasattr(m2["utils"], f)
    for name in ("Client", "FedAvg_Client", "FedProx_Client", "FedAdmm_Client"):
        assert hasattr(m["clients"], name)
    for meth in ("update_weights", "update_model", "update_duals", "inference", "train_val_test"):
        assert hasattr(m["clients"].FedAdmm_Client, meth)
    for f in ("mnist_iid", "mnist_noniid", "cifar_iid", "cifar_noniid"):
        assert hasattr(m["sampling"], f)


def test_plugin_by_name():
    m = load_project("primal_dual", ["servers", "clients"])
    s, c = m["servers"], m["clients"]
    assert s._client_class("FedAdmm_Server") is c.FedAdmm_Client
    assert s._client_class("FedProx_Server") is c.FedProx_Client
    with pytest.raises(KeyError):
        s._client_class("Scaffold_Server")


def test_dotdict_missing_keys_are_none():
    m = load_project("weighted_average", ["utils"])
    a = m["utils"].DotDict(lr=0.1)
    assert a.lr == 0.1 and a.rho is None
    a.mode = "stochastic"
    assert a["mode"] == "stochastic"


@pytest.mark.parametrize("name", ["Model1", "Model3"])
def test_model_layout_and_init_match_reference(name):
    """Same keys/shapes/P and the same default-init values under a seed
    (DIST/models.py; golden from the reference's own Model classes)."""
    from dolhip import models
    h = golden("host")
    torch.manual_seed(2028)
    m = getattr(models, name)()
    sd = m.state_dict()
    assert list(sd.keys()) == list(h[f"{name}__keys"])
    assert [str(tuple(v.shape)) for v in sd.values()] == list(h[f"{name}__shapes"])
    flat = np.concatenate([v.numpy().reshape(-1) for v in sd.values()])
    assert flat.size == int(h[f"{name}__P"][0])
    assert flat[::4999].tobytes() == h[f"{name}__sample"].tobytes()
    np.testing.assert_array_equal(
        [flat.astype(np.float64).sum(), np.abs(flat.astype(np.float64)).sum()], h[f"{name}__sum"])


class _DS:
    def __init__(self, t):
        self.targets = torch.from_numpy(t)

    def __len__(self):
        return len(self.targets)


@pytest.mark.parametrize("iid", [True, False])
def test_gossip_user_splits_match_reference(iid):
    m = load_project("weighted_average", ["sampling", "utils"])
    h = golden("host")
    ds = _DS(np.random.default_rng(5).integers(0, 10, 1200))
    np.random.seed(77)
    args = m["utils"].DotDict(num_users=6, shards=2)
    g = m["sampling"].iid_split(ds, args) if iid else m["sampling"].noniid_split(ds, args)
    for u in range(6):
        assert np.array_equal(np.array(sorted(float(i) for i in g[u])), h[f"dist_iid{iid}__u{u}"])
        if not iid:
            assert np.array_equal(np.asarray(g[u], np.float64), h[f"dist_iid{iid}__u{u}__order"])
    assert np.array_equal(np.random.random(3), h[f"dist_iid{iid}__after"])  # RNG consumed identically


def test_federated_user_splits_match_reference():
    m = load_project("primal_dual", ["sampling"])
    h = golden("host")
    ds = _DS(np.random.default_rng(5).integers(0, 10, 1200))
    np.random.seed(78)
    g = m["sampling"].mnist_iid(ds, 10)
    for u in range(10):
        assert np.array_equal(np.array(sorted(int(i) for i in g[u])), h[f"dec_iid__u{u}"])
    assert np.array_equal(np.random.random(3), h["dec_iid__after"])


def test_synthetic_data_consumes_no_global_rng():
    from dolhip.data import synthetic_pair
    np.random.seed(1)
    torch.manual_seed(1)
    synthetic_pair("synthetic", 100, 10, 3)
    a, b = np.random.random(), torch.rand(1)
    np.random.seed(1)
    torch.manual_seed(1)
    assert a == np.random.random() and torch.equal(b, torch.rand(1))


def test_no_cpu_path():
    m = load_project("weighted_average", ["clients", "utils", "models"])
    from dolhip._native import DolNativeError
    args = m["utils"].DotDict(device="cpu", local_bs=8, lr=0.1, momentum=0.5)
    with pytest.raises(DolNativeError):
        m["clients"].Client(args=args, train_set=_DS(np.zeros(20, np.int64)), test_set=_DS(np.zeros(4, np.int64)),
                            idxs=set(range(20)), model=m["models"].Model1())
