"""N>1 path rehearsed on CPU with gloo (world_size 2): per-rank sequences, max-over-ranks timing,
end-of-run gather, and bench.py's JSON contract under torch.distributed.run."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch

    from mageslam_amd import multigpu, synth

    dist = multigpu.init("gloo", rank)
    seed = multigpu.sequence_seed(synth.FRAME_SEED, rank)
    fr = synth.frame(0, 32, 24, seed)
    row = torch.tensor([[rank, int(fr.sum())]], dtype=torch.int64)
    g = multigpu.gather_rows(row, dist)
    m = multigpu.max_over_ranks(float(rank + 1), "cpu", dist)
    q.put((rank, [r.tolist() for r in g], m))
    dist.destroy_process_group()


def test_gloo_world2_gather_and_max():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29511
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, gathered, m in res:
        assert [g[0][0] for g in gathered] == [0, 1]  # ordered by rank
        assert gathered[0][0][1] != gathered[1][0][1]  # independent sequences (seed + rank)
        assert m == 2.0


def test_bench_cpu_dry_run_world2(tmp_path):
    """bench.py's N>1 flow under torch.distributed.run (gloo): per-rank sequences, max-over-ranks
    timing, and C5's exchange — every rank's trajectory all-gathered and written by rank 0 in rank
    order as ExportFossilCsv (stand-in tracking results: each rank's ground-truth poses)."""
    from mageslam_amd import synth, trajectory

    csv = tmp_path / "c5.csv"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29513", str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--cpu-dry-run", "--track-frames", "12", "--trajectory-csv", str(csv)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["gathered_ranks"] == [0, 1] and d["value"] > 0
    assert d["gathered_checksums"][0] != d["gathered_checksums"][1]
    assert d["trajectory_frames_gathered"] == 24
    # the CSV holds rank 0's sequence, then rank 1's, each exactly its own trajectory
    expect = tmp_path / "expect.csv"
    rows = []
    for rank in range(2):
        seq = synth.scene_sequence(12, 1280, 720, origin=synth.rank_origin(rank))
        rows.append(trajectory.records_from_poses(seq.R, seq.t, np.ones(12, bool)))
    trajectory.export_fossil_csv(expect, np.concatenate(rows))
    assert csv.read_text() == expect.read_text()
    assert not np.array_equal(rows[0], rows[1])


def test_fossil_csv_format(tmp_path):
    """ExportFossilCsv (console.cpp:15-54): %g-formatted view-matrix rows, identity for lost frames."""
    from mageslam_amd import trajectory

    R = np.array([[1, 0, 0], [0, 0.5, -0.866025], [0, 0.866025, 0.5]], np.float32)
    M = trajectory.view_matrices(np.float32([[0.1, -2.5, 1234567]]), R.T.reshape(1, 9))
    rows = trajectory.records([True, False], np.concatenate([M, M]))
    p = tmp_path / "mage_output.csv"
    trajectory.export_fossil_csv(p, rows)
    lines = p.read_text().splitlines()
    assert lines[0] == '"true",1,0,0,0.1,0,0.5,-0.866025,-2.5,0,0.866025,0.5,1.23457e+06,0,0,0,1'
    assert lines[1] == '"false",1,0,0,0,0,1,0,0,0,0,1,0,0,0,0,1'


def _traj_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch

    from mageslam_amd import multigpu, synth, trajectory

    dist = multigpu.init("gloo", rank)
    pb = synth.pose_batch(problems=5, obs=20, seed=multigpu.sequence_seed(synth.BA_SEED, rank))
    rows = trajectory.records(np.arange(5) != rank, trajectory.view_matrices(pb.pos, pb.r9))
    g = trajectory.gather_trajectories(torch.from_numpy(rows), dist)
    q.put((rank, [x.numpy() for x in g], rows))
    dist.destroy_process_group()


def test_gloo_world2_trajectory_gather():
    """C5's end-of-run exchange: each rank's 68-byte-per-frame trajectory, gathered in rank order."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_traj_worker, args=(r, 2, 29517, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    own = {rank: rows for rank, _, rows in res}
    for rank, gathered, _ in res:
        assert len(gathered) == 2 and gathered[0].shape == (5, 17)
        assert np.array_equal(gathered[0], own[0]) and np.array_equal(gathered[1], own[1])
    assert not np.array_equal(own[0][:, 1:], own[1][:, 1:])
