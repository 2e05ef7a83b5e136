"""bench.py's own N-rank launcher (CPU, gloo rehearsal).

``python bench.py --gpus N`` with no launcher around it must start N rank
processes itself (torch.distributed.run children; the parent makes no GPU
call), and a rank must refuse to run when the number of ranks launched is
not --gpus or when fewer GPUs are visible.  ``--rehearse`` runs the ranks
without any kernel: they form the process group, take the bench's source
shards of the k=48 fat-tree and assemble them with the bench's all-gather
helper, and rank 0 prints the line's multi-rank keys."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "BENCH_DEVICE")}
    env.update(kw)
    return env


def _run(args, env, timeout=300):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n,form", [(2, "root"), (3, "root"), (2, "all"), (2, "none")])
def test_bench_gpus_n_launches_n_ranks(n, form):
    r = _run(["--gpus", str(n), "--rehearse", "--steps", "2", "--assemble", form,
              "--cpu-budget-s", "2"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout           # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["process_group"] == {"backend": "gloo", "world_size": n}
    assert len({s["pid"] for s in line["shards"]}) == n          # n distinct processes
    assert [s["rank"] for s in line["shards"]] == list(range(n))
    # contiguous shards covering every k=48 host-bearing switch once
    assert line["shards"][0]["lo"] == 0 and line["shards"][-1]["hi"] == 1152
    assert all(a["hi"] == b["lo"] for a, b in zip(line["shards"], line["shards"][1:]))
    assert line["sources_assembled_exactly"] is True     # (none: each rank's own shard)
    # the N > 1 line's honesty keys: one step's latency, the
    # rate by steps in flight, both assembly forms preflighted, the scaling
    # efficiency against the same run's N = 1 base, why this assembly, and
    # the host-CPU baseline measured on rank 0 in the same run
    m = line["multi_gpu"]
    assert line["single_step_ms"] > 0 and m["single_step_ms"] == line["single_step_ms"]
    assert m["by_inflight"]["1"]["headline"] is True
    assert m["assembly_check"] == {"root": "ok", "all": "ok"}
    assert m["n1_base"]["inflight_1"]["value"] > 0
    assert m["scaling_efficiency"] > 0 and m["scaling_efficiency_base"] == "n1_base.inflight_1"
    assert line["config"]["assemble"] == form and line["config"]["assemble_reason"]
    cpu = line["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port"


def test_bench_refuses_world_size_mismatch():
    r = _run(["--gpus", "1", "--rehearse"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
             timeout=120)
    assert r.returncode != 0
    assert "--gpus is 1" in r.stderr


def test_bench_refuses_more_gpus_than_visible():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = _run(["--gpus", "1"], _env(), timeout=120)
    assert r.returncode != 0
    assert "GPU(s) are visible" in r.stderr


def test_pick_assembly_fallbacks():
    """The N > 1 line's assembly after the preflight: the requested form when
    it passed, the other RCCL form when only that passed, no assembly (each
    rank keeps its shard) when neither did -- the line is never lost."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    ok, bad = "ok", "error: RuntimeError('x')"
    assert b.pick_assembly("root", {"root": ok, "all": ok}) == ("root", None)
    assert b.pick_assembly("all", {"root": ok, "all": ok}) == ("all", None)
    assert b.pick_assembly("root", {"root": bad, "all": ok}) == ("all", "root -> all")
    assert b.pick_assembly("all", {"root": ok, "all": "wrong rows assembled"}) == ("root", "all -> root")
    assert b.pick_assembly("root", {"root": bad, "all": bad}) == ("none", "root -> none")
    assert b.pick_assembly("none", {"root": bad, "all": bad}) == ("none", None)
    for form in ("root", "all", "none"):
        assert b.ASSEMBLE_REASON[form]
