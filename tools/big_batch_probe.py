"""ECoG-shaped batched products on the 128x128 f32 kernel (GPU box): the Xs = C^-1 L and KL L-bar forms of
engine.py (xs_side, kl_lbar) over `nb` factors of M = 1024, timed from graph replays, beside variants that
isolate the operand layout (k-contiguous vs not) and the triangular k ranges.  Prints TFLOP/s on the
structurally nonzero work (lower tiles x their k range) and on the dense 2 M^3.
usage: python tools/big_batch_probe.py [nb] [M]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from collaborative_nonstationary_multivariate_gaussian_process_amd import hip_ops as H  # noqa: E402
from collaborative_nonstationary_multivariate_gaussian_process_amd import _lib as L  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
M = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dev = torch.device("cuda", 0)
MM = M * M
g = torch.Generator(device=dev).manual_seed(0)
A = torch.randn(nb * MM, generator=g, device=dev) / M
B = torch.randn(nb * MM, generator=g, device=dev) / M
C = torch.zeros(nb * MM, device=dev)
offs = [b * MM for b in range(nb)]
tri_work = 2.0 * M ** 3 / 3.0 * nb      # lower tiles x their k range of a triangular x triangular product
dense = 2.0 * M ** 3 * nb


def run(name, ak, bk, flags, work):
    bb = H.BigBatch(A, B, C, offs, offs, offs, M, M, M, lda=M, ldb=M, a_kcontig=ak, b_kcontig=bk, flags=flags)
    bb()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(3):
            bb()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(json.dumps({"case": name, "nb": nb, "M": M, "ms": round(ms, 3), "tflops": round(work / (ms * 1e-3) / 1e12, 2)}),
          flush=True)


run("xs_side form (A k-contig lower, B not k-contig lower, OUT_TRIL)", True, False,
    L.A_LOWER | L.B_LOWER | L.OUT_TRIL, tri_work)
run("xs form, B k-contig (B_UPPER of the transposed operand)", True, True,
    L.A_LOWER | L.B_UPPER | L.OUT_TRIL, tri_work)
run("kl_lbar form (A, B not k-contig, A_UPPER B_LOWER, OUT_TRIL)", False, False,
    L.A_UPPER | L.B_LOWER | L.OUT_TRIL, tri_work)
run("dense, both k-contig", True, True, 0, dense)
run("dense, B not k-contig", True, False, 0, dense)
run("dense, A and B not k-contig", False, False, 0, dense)
if len(sys.argv) > 3 and sys.argv[3] == "kl":
    run("kl form, A k-contig (same k ranges)", True, False, L.A_UPPER | L.B_LOWER | L.OUT_TRIL, tri_work)
    run("kl form, B k-contig (same k ranges)", False, True, L.A_UPPER | L.B_LOWER | L.OUT_TRIL, tri_work)
    run("kl form, no OUT_TRIL", False, False, L.A_UPPER | L.B_LOWER, tri_work)
    run("kl form, no triangular flags (dense k, OUT_TRIL)", False, False, L.OUT_TRIL, dense / 2)
if len(sys.argv) > 3 and sys.argv[3] == "rank":
    # the ECoG pair L-bar form: C += P^T W-hat over the ~4 rows of one output (k = 4), OUT_TRIL, beta = 1
    for kk in (4, 16, 64):
        bb = H.BigBatch(A, B, C, offs, offs, offs, M, M, kk, lda=M, ldb=M, a_kcontig=False, b_kcontig=False,
                        flags=L.OUT_TRIL, beta=1.0)
        bb()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(3):
                bb()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        # HBM floor: read + write C (lower tiles), write C (upper tiles) ~ 3/2 x 4 MB per problem
        print(json.dumps({"case": f"rank-{kk} update C += A^T B (OUT_TRIL, beta 1)", "nb": nb, "ms": round(ms, 3),
                          "GB_per_s_C_traffic": round(nb * 1.5 * M * M * 4 * 2 / 2 / (ms * 1e-3) / 1e9, 1)}),
              flush=True)
