"""hipfm — an MI355X-native DeepFM CTR training framework.

Capabilities mirror ``Chen188/deepfm-tensorflow-distributed-training-on-sagemaker``
(TF1 Estimator + Parameter-Server / Horovod DeepFM); the design is MI355X-first:

* ``hipfm.ops``       — ctypes bindings to hand-written gfx950 HIP kernels (FM fused
                         gather/interaction, MFMA MLP GEMMs with fused epilogues, fused
                         sparse-gradient reduce + row-wise optimizers, dense optimizers, AUC).
* ``hipfm.models``    — the DeepFM model: a native GPU executor (explicit fused fwd/bwd) and
                         a pure-PyTorch golden model transcribing the reference's TF1 semantics.
* ``hipfm.parallel``  — one-process-per-GPU data parallelism over RCCL (``torch.distributed``
                         backend ``nccl``): bucketed dense all-reduce overlapped with the sparse
                         backward, replicated or row-sharded embedding tables (all-to-all).
* ``hipfm.data``      — TFRecord / tf.train.Example / libsvm I/O (native C++ reader + decoder),
                         shard policy, HBM-resident batch cache, synthetic Criteo-shaped data.
* ``hipfm.ckpt``      — native checkpoints with auto-resume, TF ``tensor_bundle`` export/import,
                         servable export.
* ``hipfm.estimator`` — Estimator-style train / evaluate / predict / export and
                         ``train_and_evaluate``; ``hipfm.cli`` is the flag-compatible entrypoint.

Import as ``import hipfm`` (see ``hipfm/__init__.py`` at the repo root).
"""

__version__ = "0.1.0"
