"""Checkpoint formats: tf.js LayersModel (model.json + weights.bin), flat vars (meta.json + data.bin),
versioned directories with a ``current`` symlink and a resume record."""
from .flatvars import flat_deserialize, flat_serialize, load_flat, save_flat  # noqa: F401
from .store import VersionedStore, force_symlink  # noqa: F401
from .tfjs import (load_layers_model_weights, load_topology, read_manifest_weights,  # noqa: F401
                   save_layers_model)
