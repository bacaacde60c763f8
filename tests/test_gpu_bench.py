"""bench.py's control flow on the GPU box: one rank, and two ranks over gloo
sharing cuda:0 (the N > 1 path the driver runs over RCCL on an 8-GPU node:
the pipelined norm MAX, the collectives of every leg).  Small buckets, no
extras: this checks the JSON contract and that the pipelined issue order
gives the same packed words as the plain one, not performance."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--numel", "4000000", "--steps", "4", "--warmup", "1", "--settle", "0", "--cpu-seconds", "0", "--no-extras"]


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _check(d: dict, world: int):
    assert d["metric"] == "grad-floats/sec encode+pack (device-resident), 100M fp32 bucket; % HBM peak"
    assert d["n_gpus"] == world and d["steps"] == 4 and d["value"] > 0
    assert d["pipelined_issue_bit_identical"] is True
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["achieved"] > 0


def test_bench_one_rank():
    r = subprocess.run([sys.executable, "bench.py", *ARGS], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    _check(_line(r.stdout), 1)


def test_bench_two_ranks_gloo_pipelined():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, GC_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    _check(d, 2)
    assert d["config"]["pipelining"] and d["collectives"] == "gloo"


SCALE_ARGS = ["--numel", "2000000", "--steps", "3", "--warmup", "1", "--settle", "0", "--cpu-seconds", "0",
              "--legs", "reduce,config5", "--n5", "2000000"]


@pytest.mark.parametrize("world", [2, 4])
def test_plain_bench_gpus_n_launches_ranks(world):
    """The driver's SCALE form: plain `python bench.py --gpus N` (no torchrun,
    no WORLD_SIZE) must start N ranks itself and report them, with the
    process group's own evidence (ranks share cuda:0 over gloo here; on the
    8-GPU node the same command runs one rank per GPU over RCCL)."""
    env = dict(os.environ, GC_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(world), *SCALE_ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == world and d["config"]["parallelism"] == f"dp{world}"
    assert d["pipelined_issue_bit_identical"] is True
    pg = d["process_group"]
    assert pg["world_size"] == world and len(pg["ranks"]) == world and pg["backend"] == "gloo"
    assert sorted(x["rank"] for x in pg["ranks"]) == list(range(world))
    rp = d["reduce_path"]
    assert rp["ms_per_step"] > 0
    # per-phase HIP-event times, the packed SUM's bandwidth, the fp32 all-reduce beside it
    assert set(rp["phase_ms"]) == {"absmax", "max", "encode", "sum", "decode"}
    assert all(v >= 0 for v in rp["phase_ms"].values())
    sp, sf = rp["sum_packed"], rp["sum_fp32_reference"]
    assert sp["ms"] > 0 and sp["algbw_gbs"] > 0 and sf["ms"] > 0 and sf["bytes_per_rank"] == 4 * 2_000_000
    assert abs(sp["busbw_gbs"] - 2 * (world - 1) / world * sp["algbw_gbs"]) < 1e-6 * sp["algbw_gbs"]
    assert rp["sum_fp32_over_packed"] > 0 and rp["wire_bytes_fp32_over_packed"] > 1
    if world >= 4:
        assert d["reduce_path_2x_nodes"]["bit_identical_to_flat"] is True
    ov = d["configs"]["config5_1b_8bit_chunked"]["overlap"]
    assert ov["chunks"] == 8 and len(ov["ms"]["sum_end"]) == 8
    assert all(a <= b for a, b in zip(ov["ms"]["decode_start"], ov["ms"]["decode_end"]))
    assert len(ov["encode_c1_overlap_sum_c_ms"]) == 7 and all(v >= 0 for v in ov["encode_c1_overlap_sum_c_ms"])
    assert isinstance(ov["encode_overlaps_previous_sum"], bool)
    assert all(a <= b for a, b in zip(ov["ms"]["encode_start"], ov["ms"]["encode_end"]))


def test_bench_config5_own_lane_width_one_gpu():
    """Config 5 at its own lane width on one GPU (8-bit, lanes sized for W = 8:
    12-bit, 2 per word), with per-kernel roofline fractions."""
    args = ["--numel", "2000000", "--steps", "3", "--warmup", "1", "--settle", "0", "--cpu-seconds", "0",
            "--legs", "config5", "--n5", "3000000"]
    r = subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    c = _line(r.stdout)["configs"]["config5_1b_8bit_w8_lanes"]
    assert c["lane_bits"] == 12 and c["lanes_per_word"] == 2 and c["world_lanes"] == 8
    for k in ("k_qsgd_encode", "k_qsgd_decode"):
        assert c[k]["us"] > 0 and 0 < c[k]["frac_hbm_peak"] < 1.2
