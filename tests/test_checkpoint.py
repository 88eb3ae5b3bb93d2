"""Checkpoint formats: tf.js LayersModel (model.json + weights.bin), flat vars, versioned store."""
import json
import os

import numpy as np
import pytest
import torch

from distriflow_amd.checkpoint import (VersionedStore, load_flat, load_layers_model_weights, read_manifest_weights,
                                       save_flat, save_layers_model)
from distriflow_amd.models.distri_model import CheckpointedServerModel, DynamicServerModel, fetch_model
from distriflow_amd.models.zoo import build_model, keras_cnn_topology

REF_MODEL_JSON = "/root/reference/experiment/mnist/model.json"


def test_layers_model_round_trip(tmp_path):
    a = build_model("keras_cnn", "cpu", seed=1)
    save_layers_model(a, str(tmp_path / "m"))
    doc = json.load(open(tmp_path / "m" / "model.json"))
    assert doc["format"] == "layers-model"
    shapes = {w["name"]: w["shape"] for w in doc["weightsManifest"][0]["weights"]}
    # Keras layouts on disk, same as the reference's model.json manifest
    assert shapes["conv2d_1/kernel"] == [3, 3, 1, 32] and shapes["dense_1/kernel"] == [4608, 128]
    b = build_model("keras_cnn", "cpu", seed=2)
    load_layers_model_weights(b, str(tmp_path / "m" / "model.json"))
    assert torch.equal(a.store.master, b.store.master)
    # and the reloaded model computes the same function
    x = torch.rand(3, 28, 28, 1)
    torch.testing.assert_close(a.predict(x), b.predict(x))


def test_manifest_matches_reference_model_json(tmp_path):
    if not os.path.exists(REF_MODEL_JSON):
        pytest.skip("reference not mounted")
    ref = json.load(open(REF_MODEL_JSON))
    ref_w = [(w["name"], w["shape"]) for g in ref["weightsManifest"] for w in g["weights"]]
    net = build_model("keras_cnn", "cpu")
    save_layers_model(net, str(tmp_path / "m"), topology=ref["modelTopology"])
    ours = [(w["name"], w["shape"]) for w in json.load(open(tmp_path / "m" / "model.json"))["weightsManifest"][0]["weights"]]
    assert ours == ref_w


def test_sharded_manifest_read(tmp_path):
    net = build_model("lenet5", "cpu", seed=3)
    save_layers_model(net, str(tmp_path / "s"), shard_bytes=50000)
    files = sorted(os.listdir(tmp_path / "s"))
    assert any("shard" in f for f in files)
    w = read_manifest_weights(str(tmp_path / "s" / "model.json"))
    np.testing.assert_array_equal(w["dense_1/kernel"], net.store["dense_1/kernel"].t().numpy())


def test_fetch_model_from_reference_topology():
    net = fetch_model(REF_MODEL_JSON if os.path.exists(REF_MODEL_JSON) else "keras_cnn", device="cpu")
    assert net.num_params() == 600165


def test_flat_vars_round_trip(tmp_path):
    vs = [torch.randn(3, 4), torch.arange(5, dtype=torch.int32), torch.tensor([True, False])]
    save_flat(str(tmp_path / "f"), vs)
    meta = json.load(open(tmp_path / "f" / "meta.json"))
    assert meta["byteOffsets"] == [0, 48, 68]
    back = load_flat(str(tmp_path / "f"))
    assert all(torch.equal(a, b) for a, b in zip(vs, back))


def test_versioned_store(tmp_path):
    st = VersionedStore(str(tmp_path / "v"), keep_last=2)
    st.setup()
    vs = []
    for _ in range(4):
        v = st.new_version()
        os.makedirs(st.path(v))
        st.mark_current(v)
        vs.append(v)
        st.prune()
    assert vs == sorted(vs, key=int) and len(set(vs)) == 4  # strictly increasing, no ms collisions
    assert st.list() == vs[-2:] and st.current() == vs[-1] and st.last() == vs[-1]
    st.write_resume({"epoch": 3})
    assert st.read_resume() == {"epoch": 3}


def test_checkpointed_server_model_resumes(tmp_path):
    m = CheckpointedServerModel(str(tmp_path / "ck"), "mlp_mnist", device="cpu")
    m.setup()
    v0 = m.version
    m.net.store.grad.fill_(0.5)
    m.update_flat(m.net.store.grad)
    m.save()
    assert m.version != v0 and os.path.islink(tmp_path / "ck" / "current")
    m2 = CheckpointedServerModel(str(tmp_path / "ck"), "mlp_mnist", device="cpu")
    m2.setup()
    assert m2.version == m.version
    assert torch.equal(m2.get_flat(), m.get_flat())


def test_dynamic_server_model_load_assigns(tmp_path):
    w = [torch.ones(2, 2), torch.zeros(3)]
    m = DynamicServerModel(str(tmp_path / "d"), w, lambda x: x, lambda y, p: (y - p) ** 2, [1], [1])
    m.setup()
    m.set_vars([torch.full((2, 2), 3.0), torch.ones(3)])
    m.save()
    m2 = DynamicServerModel(str(tmp_path / "d"), w, lambda x: x, lambda y, p: (y - p) ** 2, [1], [1])
    m2.setup()
    assert torch.equal(m2.get_vars()[0], torch.full((2, 2), 3.0))
