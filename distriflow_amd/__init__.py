"""distriflow_amd — an MI355X-native data-parallel training framework with the capabilities of
Christopher-Wang/DistriFlow (TypeScript / tensorflow.js parameter-server library).

Public API (reference barrel: /root/reference/src/index.ts -> client / common / server):

* roles      DistriServer / FederatedServer (sync FedSGD), AsynchronousSGDServer (bounded staleness),
             FedAvgServer; DistriWorker / FederatedClient, AsynchronousSGDClient, FedAvgClient
* data par.  DataParallelTrainer — RCCL all-reduce synchronous SGD over xGMI (headline benchmark)
* models     DistriModel, EngineModel (DistributedTfModel), DynamicModel, server/client models,
             Net + layers + model zoo (mlp_mnist, keras_cnn, lenet5, resnet18_cifar)
* data       DistriDataset (FCFS microbatch dispenser), synthetic / IDX MNIST loaders
* protocol   SerializedVariable, serialize/deserialize/stack, message types, Events
* config     reference defaults + override semantics
* checkpoint tf.js LayersModel format, flat-vars format, versioned store + resume record

Heavy submodules are imported lazily so ``import distriflow_amd`` stays cheap.
"""
from __future__ import annotations

import importlib

__version__ = "0.1.0"

_LAZY = {
    # config / protocol
    "DEFAULT_CLIENT_HYPERPARAMS": "config", "DEFAULT_SERVER_HYPERPARAMS": "config",
    "DEFAULT_DATASET_HYPERPARAMS": "config", "DEFAULT_DISTRIBUTED_COMPILE_ARGS": "config",
    "client_hyperparams": "config", "server_hyperparams": "config", "override": "config",
    "SerializedVariable": "protocol", "serialize_var": "protocol", "serialize_vars": "protocol",
    "deserialize_var": "protocol", "deserialize_vars": "protocol", "stack_serialized": "protocol",
    "Events": "protocol", "ModelMsg": "protocol", "GradientMsg": "protocol", "DataMsg": "protocol",
    "UploadMsg": "protocol", "DownloadMsg": "protocol",
    "LOSSES": "losses", "lossesMap": "losses",
    # models
    "Net": "models.net", "build_model": "models.zoo", "MODELS": "models.zoo",
    "DistriModel": "models.distri_model", "EngineModel": "models.distri_model",
    "DynamicModel": "models.distri_model", "InMemoryServerModel": "models.distri_model",
    "CheckpointedServerModel": "models.distri_model", "DynamicServerModel": "models.distri_model",
    "ClientModel": "models.distri_model", "fetch_model": "models.distri_model",
    "DistributedModel": "models.distri_model", "DistributedTfModel": "models.distri_model",
    "DistributedDynamicModel": "models.distri_model", "DistributedServerInMemoryModel": "models.distri_model",
    "DistributedServerTfModel": "models.distri_model", "DistributedServerDynamicModel": "models.distri_model",
    "DistributedClientTfModel": "models.distri_model", "MockModel": "models.mock",
    # data
    "DistriDataset": "data.dataset", "DistributedDataset": "data.dataset", "Batch": "data.dataset",
    "batch_to_data_msg": "data.dataset", "batchToDataMSG": "data.dataset",
    # roles / parallel
    "AbstractServer": "parallel.server", "FederatedServer": "parallel.server", "DistriServer": "parallel.server",
    "AsynchronousSGDServer": "parallel.server", "FedAvgServer": "parallel.server",
    "AbstractWorker": "parallel.worker", "FederatedClient": "parallel.worker", "DistriWorker": "parallel.worker",
    "AsynchronousSGDClient": "parallel.worker", "FedAvgClient": "parallel.worker",
    "LocalHub": "parallel.transport", "DistTransport": "parallel.transport",
    "DataParallelTrainer": "parallel.data_parallel", "init_distributed": "parallel.comm",
}


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError(f"module 'distriflow_amd' has no attribute {name!r}")
    return getattr(importlib.import_module(f".{mod}", __name__), name)


def __dir__():
    return sorted(list(globals()) + list(_LAZY))
