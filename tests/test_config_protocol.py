"""Config defaults/override semantics and the wire protocol (reference serialization_test.ts)."""
import pytest
import torch

from distriflow_amd import config as C
from distriflow_amd import protocol as P


def test_defaults_match_reference():
    assert C.DEFAULT_CLIENT_HYPERPARAMS == {"examplesPerUpdate": 5, "learningRate": 0.001, "batchSize": 32, "epochs": 5}
    assert C.DEFAULT_SERVER_HYPERPARAMS["aggregation"] == "mean"
    assert C.DEFAULT_SERVER_HYPERPARAMS["minUpdatesPerVersion"] == 20
    assert C.DEFAULT_DATASET_HYPERPARAMS == {"batchSize": 32, "epochs": 5, "smallLastBatch": False}
    assert C.DEFAULT_DISTRIBUTED_COMPILE_ARGS["loss"] == "meanSquaredError"


def test_override_reference_semantics():
    out = C.override(C.DEFAULT_CLIENT_HYPERPARAMS, {"examplesPerUpdate": 1, "learningRate": 0})
    assert out["examplesPerUpdate"] == 1
    assert out["learningRate"] == 0.001  # falsy -> default (reference quirk)
    with pytest.raises(ValueError, match="Unrecognized key"):
        C.override(C.DEFAULT_CLIENT_HYPERPARAMS, {"bogus": 1})
    assert C.strict_override(C.DEFAULT_CLIENT_HYPERPARAMS, {"learning_rate": 0})["learningRate"] == 0


def test_hyperparam_helpers_and_env(monkeypatch):
    with pytest.raises(ValueError, match="clientHyperparams"):
        C.client_hyperparams({"nope": 3})
    monkeypatch.setenv("DISTRIFLOW_MIN_UPDATES_PER_VERSION", "4")
    assert C.server_hyperparams({})["minUpdatesPerVersion"] == 4
    monkeypatch.setenv("DISTRIFLOW_SERVER_MIN_UPDATES_PER_VERSION", "7")
    assert C.server_hyperparams({})["minUpdatesPerVersion"] == 7


def test_serialize_round_trip():
    cases = [torch.arange(8, dtype=torch.float32).view(2, 2, 2), torch.tensor([True, False, True]),
             torch.arange(6, dtype=torch.int32).view(2, 3), torch.randn(5).to(torch.bfloat16)]
    for t in cases:
        s = P.serialize_var(t)
        assert s.dtype == P.dtype_name(t.dtype) and s.shape == list(t.shape)
        back = P.deserialize_var(s)
        assert back.dtype == t.dtype and torch.equal(back, t)


def test_stack_serialized():
    ups = [[P.serialize_var(torch.full((2, 2, 2), float(u))), P.serialize_var(torch.full((2, 2), u, dtype=torch.int32))]
           for u in range(3)]
    st = P.stack_serialized(ups)
    assert st[0].shape == [3, 2, 2, 2] and st[0].dtype == "float32"
    assert st[1].shape == [3, 2, 2] and st[1].dtype == "int32"
    a = P.deserialize_var(st[0])
    assert torch.equal(a[2], torch.full((2, 2, 2), 2.0))


def test_header_round_trip():
    pl = [torch.zeros(10), torch.zeros(3, dtype=torch.int64)]
    h = P.encode_header(P.Kind.UPLOAD, 3, version_id=7, batch=5, epoch=1, metrics=[0.5, 0.25], num_examples=32,
                        payloads=pl)
    d = P.decode_header(h)
    assert d["kind"] == P.Kind.UPLOAD and d["src"] == 3 and d["version_id"] == 7 and d["batch"] == 5
    assert d["metrics"] == [0.5, 0.25] and d["num_examples"] == 32
    assert d["payloads"] == [(torch.float32, 10), (torch.int64, 3)]
    assert P.payload_json(P.json_payload({"a": [1, 2]})) == {"a": [1, 2]}


def test_client_buffer_utils():
    """Reference src/client/utils.ts:22-47 (concat/slice with empty tensors, addRows single or batch)."""
    import pytest as _pytest

    from distriflow_amd.utils.tensors import add_rows, concat_with_empty, slice_with_empty, wait_for

    e = torch.empty(0, 2, 2)
    one = torch.ones(2, 2)
    b = add_rows(e, one, (2, 2))
    assert b.shape == (1, 2, 2)
    b = add_rows(b, torch.zeros(3, 2, 2), (2, 2))
    assert b.shape == (4, 2, 2) and b[0].sum() == 4
    with _pytest.raises(ValueError):
        add_rows(b, torch.zeros(3, 3), (2, 2))
    assert concat_with_empty(e, b).shape == (4, 2, 2) and concat_with_empty(b, e).shape == (4, 2, 2)
    assert slice_with_empty(b, 3).shape == (1, 2, 2) and slice_with_empty(b, 9).shape == (0, 2, 2)
    assert slice_with_empty(b, 1, 2).shape == (2, 2, 2)
    hits = iter([None, None, 7])
    assert wait_for(lambda: next(hits), timeout=1.0) == 7
    with _pytest.raises(TimeoutError):
        wait_for(lambda: None, timeout=0.01)
