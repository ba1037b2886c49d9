"""Route tables and lane layout of the Python layer (reference utils.py:1-98).

Kept for drop-in compatibility: env.py stores the Python lane layout and uses
the default route mappings to pick ego routes and the NPC route list.  As in
the reference, the Python layout uses a 900x900 canvas (reference utils.py:4)
that is only stored, never sent to the simulator (which works on 750x750).
"""
from __future__ import annotations

from typing import Dict, List

# reference utils.py:4-8 (the Python side's canvas; the simulator's is 750x750)
WIDTH, HEIGHT = 900, 900
SCALE = 12
LANE_WIDTH_M = 3.5
LANE_WIDTH_PX = int(LANE_WIDTH_M * SCALE)
OBS_DIM = 127

# reference utils.py:15-27
DEFAULT_REWARD_CONFIG = {
    "use_team_reward": False,
    "traffic_flow": False,
    "reward_config": {
        "progress_scale": 10.0,
        "stuck_speed_threshold": 1.0,
        "stuck_penalty": -0.01,
        "crash_vehicle_penalty": -10.0,
        "crash_object_penalty": -5.0,
        "success_reward": 10.0,
        "action_smoothness_scale": -0.02,
        "team_alpha": 0.2,
    },
}


def _mapping(pairs) -> Dict[str, List[str]]:
    return {f"IN_{s}": [f"OUT_{e}"] for s, e in pairs}


# reference utils.py:29-52 (start lane -> [end lanes])
DEFAULT_ROUTE_MAPPING_2LANES = _mapping([(1, 3), (2, 6), (3, 5), (4, 8), (6, 2), (7, 1), (8, 4)])
DEFAULT_ROUTE_MAPPING_3LANES = _mapping([(1, 4), (2, 8), (3, 12), (4, 7), (5, 11), (6, 3),
                                         (7, 10), (8, 2), (9, 6), (10, 1), (11, 5), (12, 9)])


def build_lane_layout(num_lanes: int) -> dict:
    """Lane entry/exit points on the Python 900x900 canvas (reference utils.py:55-98)."""
    dir_order = ["N", "E", "S", "W"]
    points, in_by_dir, out_by_dir, dir_of, idx_of = {}, {d: [] for d in dir_order}, {d: [] for d in dir_order}, {}, {}
    margin = 30
    cx, cy = WIDTH // 2, HEIGHT // 2
    for d_idx, d in enumerate(dir_order):
        for j in range(num_lanes):
            off = LANE_WIDTH_PX * (0.5 + j)
            k = d_idx * num_lanes + j + 1
            i_name, o_name = f"IN_{k}", f"OUT_{k}"
            if d == "N":
                points[i_name], points[o_name] = (cx - off, margin), (cx + off, margin)
            elif d == "S":
                points[i_name], points[o_name] = (cx + off, HEIGHT - margin), (cx - off, HEIGHT - margin)
            elif d == "E":
                points[i_name], points[o_name] = (WIDTH - margin, cy - off), (WIDTH - margin, cy + off)
            else:
                points[i_name], points[o_name] = (margin, cy + off), (margin, cy - off)
            in_by_dir[d].append(i_name)
            out_by_dir[d].append(o_name)
            dir_of[i_name] = dir_of[o_name] = d
            idx_of[i_name] = idx_of[o_name] = j
    return {"points": points, "in_by_dir": in_by_dir, "out_by_dir": out_by_dir, "dir_of": dir_of,
            "idx_of": idx_of, "dir_order": dir_order}


def default_routes(num_lanes: int) -> List[tuple]:
    """All (start, end) pairs of the default mapping, in mapping order (env.py:138-145)."""
    mapping = DEFAULT_ROUTE_MAPPING_2LANES if num_lanes == 2 else DEFAULT_ROUTE_MAPPING_3LANES
    return [(s, e) for s, ends in mapping.items() for e in ends]


def point_index(name: str, num_lanes: int) -> int:
    """Lane-point name -> C-ABI point index ("IN_k" -> k-1, "OUT_k" -> 4L+k-1); -1 if unknown."""
    try:
        kind, k = name.split("_")
        k = int(k)
    except (ValueError, AttributeError):
        return -1
    if not 1 <= k <= 4 * num_lanes or kind not in ("IN", "OUT"):
        return -1
    return k - 1 if kind == "IN" else 4 * num_lanes + k - 1


def point_name(idx: int, num_lanes: int) -> str:
    return f"IN_{idx + 1}" if idx < 4 * num_lanes else f"OUT_{idx - 4 * num_lanes + 1}"
