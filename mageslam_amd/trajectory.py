"""Trajectory output — the per-frame tracking results the C5 configuration gathers across ranks and
the CSV the reference's console app writes (Apps/Console/console.cpp:15-54 ExportFossilCsv, from
MAGESlam::FossilizedMap::GetTrackingResultsForFrames, Core/MAGESLAM/Source/MAGESlam.cpp:410-428).

A frame's record is 17 float32 (68 bytes): tracked flag + the 4x4 view matrix M11..M44 row-major
([R | t; 0 0 0 1], t = view-space position, as Pose::GetViewMatrix).
"""
from __future__ import annotations

import numpy as np

RECORD_FLOATS = 17


def view_matrices(pos3: np.ndarray, r9_colmajor: np.ndarray) -> np.ndarray:
    """(T, 4, 4) float32 view matrices from BundlerLib::GetPose outputs (t, column-major R)."""
    pos3 = np.asarray(pos3, np.float32).reshape(-1, 3)
    R = np.asarray(r9_colmajor, np.float32).reshape(-1, 3, 3).transpose(0, 2, 1)
    M = np.zeros((len(pos3), 4, 4), np.float32)
    M[:, :3, :3] = R
    M[:, :3, 3] = pos3
    M[:, 3, 3] = 1
    return M


def records(tracked: np.ndarray, mats: np.ndarray) -> np.ndarray:
    """(T, 17) float32 rows: flag, then M11..M44."""
    tracked = np.asarray(tracked, bool).reshape(-1)
    out = np.zeros((len(tracked), RECORD_FLOATS), np.float32)
    out[:, 0] = tracked
    out[:, 1:] = np.asarray(mats, np.float32).reshape(-1, 16)
    return out


def records_from_poses(R: np.ndarray, t: np.ndarray, tracked) -> np.ndarray:
    """(T, 17) float32 rows from per-frame world -> camera rotations (T, 3, 3) and view-space
    translations (T, 3) (the tracker's Pose, as GetTrackingResultsForFrames reports it)."""
    R = np.asarray(R, np.float64).reshape(-1, 3, 3)
    M = np.zeros((len(R), 4, 4), np.float32)
    M[:, :3, :3] = R
    M[:, :3, 3] = np.asarray(t, np.float64).reshape(-1, 3)
    M[:, 3, 3] = 1
    return records(tracked, M)


def gather_trajectories(rows, dist):
    """All-gather every rank's (T, 17) record tensor (RCCL over xGMI on GPU, gloo in tests);
    returns the list ordered by rank — the one exchange of the C5 configuration."""
    from . import multigpu

    return multigpu.gather_rows(rows, dist)


def _fmt(v: float) -> str:
    # std::ostream << float: %g with the default precision 6
    return format(float(v), "g")


def export_fossil_csv(path, rows: np.ndarray) -> None:
    """ExportFossilCsv (console.cpp:15-54): one line per frame, "true" + the 16 matrix entries, or
    the identity with "false" for untracked frames."""
    rows = np.asarray(rows, np.float32).reshape(-1, RECORD_FLOATS)
    with open(path, "w", newline="\n") as f:
        for r in rows:
            if r[0] != 0:
                f.write('"true",' + ",".join(_fmt(v) for v in r[1:]) + "\n")
            else:
                f.write('"false",1,0,0,0,0,1,0,0,0,0,1,0,0,0,0,1\n')
