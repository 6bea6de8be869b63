"""Every ``HIPFM_*`` environment knob, in one registry.

The production path needs none of them: each default is the measured-best configuration.  Kinds:

* ``variant`` -- selects an unfused / alternative execution path.  Each variant is kept because a
  test uses it as the bitwise (or tolerance) oracle of the fused path, or because it is the
  fallback of a fused path with a shape limit; the fused default is what ``bench.py`` measures.
* ``tuning``  -- a launch-shape number; the comment says what it was measured against.
* ``harness`` -- build / test / benchmark plumbing (library path, fault injection, the bench
  supervisor's protocol between parent and child processes).

``knob(name)`` returns the environment value or the registered default; reading an unregistered
name raises, and ``tests/test_knobs.py`` checks that every ``HIPFM_*`` name in the sources is
registered here, so a new switch cannot appear without its entry.
"""
from __future__ import annotations

import os
from typing import Dict, NamedTuple, Optional


class Knob(NamedTuple):
    default: Optional[str]
    kind: str
    doc: str


KNOBS: Dict[str, Knob] = {
    # ---- execution-path variants (oracles / fallbacks of the fused defaults)
    "HIPFM_SORT": Knob("auto", "variant", "auto: per-field LDS sort when field id ranges are known; "
                       "global: the 3-pass global radix sort (oracle of the field sort)"),
    "HIPFM_SORT_SIDE_STREAM": Knob("1", "variant", "slot sort on a graph side branch (0: inline)"),
    "HIPFM_SPARSE": Knob("fused", "variant", "fused: one-launch sparse backward; seg: fm_bwd_seg + "
                         "seg_apply (oracle, tests/test_gpu_kernels.py)"),
    "HIPFM_SHARD_PIPELINE": Knob("1", "variant", "row-sharded step: next batch's routing on a side "
                                 "stream (0: inline)"),
    "HIPFM_FUSED_TOWER": Knob("1", "variant", "one-launch deep tower (0: per-layer GEMM kernels)"),
    "HIPFM_TOWER_GATHER": Knob("1", "variant", "FM gather in the tower's prologue (0: fm_fwd launch)"),
    "HIPFM_WGFIN": Knob("1", "variant", "weight gradients + combine + dense optimizer in one launch "
                        "(0: wgrad_group + finalize)"),
    "HIPFM_SFWG": Knob("1", "variant", "wgfin work inside the sparse backward's launch"),
    "HIPFM_RUN_SORT": Knob("1", "variant", "multi-step graphs: every batch of the run sorted (one GPU) "
                           "or sorted + routed + its ids exchanged (row-sharded) at the graph's start "
                           "(0: the next batch's sort / routing on a side branch of each step, the "
                           "oracle and the bench ladder's second rung)"),
    "HIPFM_SH_APPLY_DENSE": Knob("1", "variant", "row-sharded step: dense optimizer in the owner "
                                 "update's launch"),
    "HIPFM_DENSE_XCHG": Knob("allgather", "variant", "fused multi-rank exchange: the dense gradient "
                             "all-gathered and summed in rank order by the owner launch (allgather: the "
                             "default, deterministic, 7 x 0.2 MB per rank at N = 8) or all-reduced by RCCL "
                             "(allreduce; auto: all-reduce from 4 ranks -- both reassociate the sum)"),
    "HIPFM_SH_OVERLAP": Knob("0", "variant", "multi-rank step (lazy or the tf1_dense split form): the dense gradient in its own "
                             "launch after the tower, all-reduced on the main stream while the sparse "
                             "backward runs on a graph branch (1), instead of all-gathered with the "
                             "gradient rows after it (0: one queue, no join; the 1-rank proxy's best)"),
    "HIPFM_SH_ROUTE2": Knob("1", "variant", "two-launch routing (0: segments + bucket kernels, oracle)"),
    "HIPFM_GROW": Knob("1", "variant", "run-sorted steps: the tower writes per-slot gradient rows, 1 at "
                       "their sorted positions (streamed), 2 in slot order (gathered through perm); 0: the "
                       "sparse launch gathers dX0 / S / vals / dlogit per slot"),
    "HIPFM_DX0_SPLIT": Knob("auto", "variant", "the tower's dX0 phase in a launch of its own: auto (batches "
                            "below 4096 rows, where the tower has < 128 blocks) | 1 | 0"),
    "HIPFM_L0_SPLIT": Knob("auto", "variant", "the fused tower's FM gather + layer 0 over ~8 field slices "
                           "in a launch of their own (auto: with the dX0 split, batches below 4096 rows) | 0"),
    "HIPFM_XROWS": Knob("fp32", "variant", "row-sharded exchange rows: fp32 (48 B at K = 8, bitwise the "
                        "one-GPU reads: the default, numerically the single-GPU step) | bf16 (opt-in: v as "
                        "bf16 + fp32 w, 24 B; fused gather tower; the FM terms then read bf16-rounded v)"),
    "HIPFM_WIRE_COMPACT": Knob("1", "variant", "streamed input: a batch ships only the value columns of "
                               "fields not all 1.0 (expanded on the device; lossless) | 0: full [B, F] values"),
    "HIPFM_GPU_DECODE": Knob("1", "variant", "streamed TFRecord epochs: the loader only frames records (length "
                             "CRC) and ships their Example bytes with their data CRCs; the GPU verifies the "
                             "CRCs and decodes into the ring slot (csrc/kernels/decode.hip) | 2: GPU decode, "
                             "data CRCs on the host | 0: host decode + compact wire"),
    "HIPFM_ASM_RING": Knob("1", "variant", "streamed input: the loader's C++ assembler thread fills the "
                           "pinned buffers ahead of the copy-issuing thread (0: that thread assembles "
                           "each batch itself, next_into)"),
    "HIPFM_TF1_SPLIT": Knob("1", "variant", "tf1_dense on one GPU: split form (0: gradient scatter + "
                            "full-table sweep, the oracle in tests/test_gpu_tf1.py)"),
    "HIPFM_SWEEP_MODE": Knob("auto", "variant", "tf1_dense split sweep: merged (workgroups of the "
                             "sparse launch) | branch (own graph branch) | auto (merged from B = 8192: "
                             "B=16384 0.156 vs 0.160-0.163 ms, B=1024 0.077 vs 0.069 ms)"),
    "HIPFM_LDS_GEMM": Knob("1", "variant", "per-layer tower GEMMs with >= 256 128x128 output tiles on the "
                           "LDS-staged workgroup tile (mlp.hip gemm_lds_kernel); 0: the register-fed "
                           "32-row tiles (bitwise the same sums: tests/test_gpu_gemm.py)"),
    "HIPFM_WG_DIRECT": Knob("1", "variant", "per-layer weight-gradient GEMMs on the 256x256 ping-pong "
                            "tile with >= 256 output tiles run unsplit and store straight into the flat "
                            "gradient (no slab, no finalize job); 0: split-K slabs summed by finalize"),
    "HIPFM_WG_BLAS": Knob("1", "variant", "the unsplit wide weight gradients (HIPFM_WG_DIRECT) as a plain "
                          "library GEMM (torch.mm bf16 -> fp32 out, hipBLASLt) into the flat gradient -- no "
                          "epilogue to fuse there (4096x3 tower 4.28 -> 3.98 ms/step, same losses: "
                          "profiles/r6_wgrad_blas_ab.log); 0: the 256x256 ping-pong tile"),
    "HIPFM_EPI_BLAS": Knob("1", "variant", "wide per-layer forward / dgrad GEMMs (256x256 ping-pong shapes, "
                           "reduction >= 1024) as a library GEMM (torch.mm, fp32 out) + the stand-alone "
                           "epilogue pass (mlp.hip epi_pass_kernel): 4096x3 tower 3.89-3.91 -> 3.49-3.50 "
                           "ms/step, bitwise the same losses (profiles/r6_epi_blas_ab.log); 0: the "
                           "fused-epilogue ping-pong tile (0.63-0.66x hipBLASLt)"),
    "HIPFM_DX0_BLAS": Knob("1", "variant", "per-layer wide tower (first layer >= 1024 units): dX0 (unmasked "
                           "bf16 product) as a library GEMM with a bf16 result, 58 vs 81 us at 16384x384x4096, "
                           "same losses (profiles/r6_dx0_blas_ab.log); 0: the LDS tile"),
    "HIPFM_TABLE_LAYOUT": Knob("record", "variant", "record: one 128-B record per row (v, w, slots); "
                               "split: separate tables"),
    # ---- tuning
    "HIPFM_FSORT_PB": Knob(None, "tuning", "field sort MSD partitions per field, log2 (default: 0 on "
                           "one GPU, 2 for the sharded routing)"),
    "HIPFM_FS_MAX_PB": Knob("4", "tuning", "tools/bench_sort.py: field sort partitions per field"),
    "HIPFM_H2D_STREAMS": Knob("2", "tuning", "streamed input: copy streams the device-ring batches alternate over"),
    "HIPFM_RAW_ROW_BYTES": Knob("2048", "tuning", "GPU decode: staging bytes per row of a batch's raw records "
                                "(a larger batch fails loudly; Criteo-shape Examples are ~330 B)"),
    "HIPFM_GRAPH_STEPS": Knob("32", "tuning", "most training steps per captured HIP graph (bench.py)"),
    # ---- harness
    "HIPFM_SAME_DEVICE": Knob("0", "harness", "multi-rank runs with every rank on device 0: gloo process "
                              "group + the same-device collective engine (parallel/loopback.py) -- the "
                              "N-GPU job's processes and step rehearsed on one GPU"),
    "HIPFM_SAME_DEVICE_CU_SPLIT": Knob("1", "harness", "same-device rehearsal: each rank's queues get a disjoint "
                                      "slice of the CUs (ROC_GLOBAL_CU_MASK; 0: every rank on every CU)"),
    "HIPFM_LB_TIMEOUT_MS": Knob("60000", "harness", "same-device engine: a collective barrier waits at "
                                "most this long, then poisons the transport (every rank raises)"),
    "HIPFM_ARCH": Knob("gfx950", "harness", "offload arch of the HIP build"),
    "HIPFM_KERNELS_SO": Knob(None, "harness", "path of the kernel library (default: in-tree _lib)"),
    "HIPFM_BUILD_PACKED": Knob(None, "harness", "build: packed-FP32 ops on (own objects / library)"),
    "HIPFM_BUILD_VARIANT": Knob(None, "harness", "build: diagnostic variant <tag>:<DEF>,<DEF> (own objects / library)"),
    "HIPFM_BUILD_STAMPS": Knob(None, "harness", "build: per-workgroup phase stamps (own objects / library)"),
    "HIPFM_BENCH_FM_IDS": Knob(None, "harness", "bench: resident batches' ids stored field-major (= --field_major_ids)"),
    "HIPFM_BENCH_STAMPS": Knob(None, "harness", "bench: save the stamp build's phase stamps (.npz path)"),
    "HIPFM_PIPE_ROOT": Knob(None, "harness", "directory of SageMaker pipe-mode FIFOs (tests)"),
    "HIPFM_FAULT_STEP": Knob(None, "harness", "fault injection: step at which a rank dies"),
    "HIPFM_FAULT_RANK": Knob(None, "harness", "fault injection: the rank (default all)"),
    "HIPFM_FAULT_MODE": Knob("exit", "harness", "fault injection: exit | raise"),
    "HIPFM_PROFILE_STEPS": Knob("", "harness", "a:b -- roctx range around steps [a, b)"),
    "HIPFM_OS_DEBUG_NOLB": Knob(None, "harness", "onesweep sort debug: disable the look-back"),
    "HIPFM_BENCH_CHILD": Knob(None, "harness", "bench supervisor protocol: set in the child"),
    "HIPFM_BENCH_SUPERVISE": Knob(None, "harness", "bench supervisor protocol: 0 runs unsupervised"),
    "HIPFM_BENCH_RUNG": Knob(None, "harness", "bench supervisor protocol: the child's ladder rung"),
    "HIPFM_BENCH_FIRST_RUNG": Knob(None, "harness", "bench: start the ladder at this rung"),
    "HIPFM_BENCH_HANG_S": Knob(None, "harness", "bench: seconds without progress = hung (45)"),
    "HIPFM_BENCH_FIRST_S": Knob(None, "harness", "bench: seconds to a rung's first progress mark (90)"),
    "HIPFM_BENCH_XGRAPH": Knob(None, "harness", "bench: most steps per captured multi-rank graph (32)"),
    "HIPFM_BENCH_NO_GRAPH": Knob(None, "harness", "bench: eager steps only"),
    "HIPFM_BENCH_DIAG": Knob(None, "harness", "bench: after the measurement, re-time the window after "
                             "idle gaps (stderr; diagnostics only)"),
    "HIPFM_BENCH_PROGRESS": Knob(None, "harness", "bench supervisor protocol: progress file"),
    "HIPFM_BENCH_RESULT": Knob(None, "harness", "bench supervisor protocol: result file"),
    "HIPFM_BENCH_FAKE": Knob(None, "harness", "bench supervisor tests: CPU stand-in children"),
}


def knob(name: str) -> Optional[str]:
    """The environment value of a registered knob, else its default."""
    k = KNOBS[name]
    return os.environ.get(name, k.default)


def flag(name: str) -> bool:
    """A registered on/off knob ("1" = on)."""
    return knob(name) == "1"


def describe() -> str:
    """One line per knob (README / ``python -m hipfm.utils.knobs``)."""
    return "\n".join(f"{n:26s} {k.kind:8s} default={k.default!s:8s} {k.doc}" for n, k in KNOBS.items())


if __name__ == "__main__":
    print(describe())
