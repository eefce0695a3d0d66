"""Camera-per-GPU sharding of a MultiFrame and the cMultiFrame concatenation.

Reference: cMultiFrame ctor, src/cMultiFrame.cpp:92-216. It extracts the cameras of one
MultiFrame in parallel (`#pragma omp parallel for num_threads(nrCams)`, :128; one extractor
per camera, :138-139), then concatenates them in camera order into mvKeys with the maps
keypoint_to_cam / cont_idx_to_local_cam_idx (:166-184), and assigns grid cells with PosInGrid
(:342-353; FRAME_GRID_COLS 64 x FRAME_GRID_ROWS 48, include/cMultiFrame.h:47-48).

MI355X mapping: camera c lives on rank c % world (slot c // world)
and is extracted there. The extractor writes fixed-capacity per-camera blocks (count,
keypoints, descriptors). One all-gather per buffer (RCCL over xGMI when the backend is nccl,
gloo in the CPU tests) replaces the shared-memory hand-off of the OpenMP threads. The
concatenation below then runs on every rank in camera order.
"""
import numpy as np

FRAME_GRID_COLS = 64
FRAME_GRID_ROWS = 48


def owned_cameras(ncams, world, rank):
    """Cameras extracted on `rank` (round-robin, so 8 cameras on 8 GPUs = one each)."""
    return [c for c in range(ncams) if c % world == rank]


def slots_per_rank(ncams, world):
    return -(-ncams // world)


def camera_order_index(ncams, world):
    """Row of camera c in the gathered [world * S] block array (rank-major)."""
    S = slots_per_rank(ncams, world)
    return [(c % world) * S + c // world for c in range(ncams)]


def gather_camera_blocks(local, ncams, group=None):
    """All-gather per-camera blocks.

    local: torch tensor [S, ...] -- this rank's owned cameras in slot order, padded to
    S = ceil(ncams / world) slots (pad rows are ignored).  Returns [ncams, ...] in camera
    order on every rank.  The one exchange step of the sharded front-end.
    """
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local[:ncams]
    world = dist.get_world_size(group)
    S = slots_per_rank(ncams, world)
    if local.shape[0] != S:
        raise ValueError("local block has %d slots, expected %d" % (local.shape[0], S))
    local = local.contiguous()
    out = torch.empty((world * S,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), local, group=group)
    idx = torch.tensor(camera_order_index(ncams, world), device=local.device)
    return out.index_select(0, idx)


def concat_multiframe(counts, kps, desc):
    """cMultiFrame concatenation (:166-184).

    counts [C] int, kps [C, cap] KEYPOINT_DTYPE (or [C, cap, 7] int32 words), desc
    [C, cap, B] u8.  Returns dict with mvKeys (sum N_c), keypoint_to_cam, cont_idx_to_local,
    descriptors (list of [N_c, B] per camera, like mDescriptors[c]) and N per camera.
    """
    from . import KEYPOINT_DTYPE
    counts = np.asarray(counts).astype(np.int64)
    kps = np.asarray(kps)
    if kps.dtype != KEYPOINT_DTYPE:
        kps = np.ascontiguousarray(kps).view(KEYPOINT_DTYPE).reshape(kps.shape[0], -1)
    C = len(counts)
    keys = np.concatenate([kps[c, :counts[c]] for c in range(C)]) if C else \
        np.zeros(0, KEYPOINT_DTYPE)
    k2c = np.concatenate([np.full(counts[c], c, np.int32) for c in range(C)]) if C else \
        np.zeros(0, np.int32)
    k2l = np.concatenate([np.arange(counts[c], dtype=np.int32) for c in range(C)]) if C else \
        np.zeros(0, np.int32)
    descs = [np.asarray(desc[c, :counts[c]]) for c in range(C)]
    return {"mvKeys": keys, "keypoint_to_cam": k2c, "cont_idx_to_local_cam_idx": k2l,
            "descriptors": descs, "N": counts.astype(np.int32)}


def grid_positions(x, y, width, height, min_x=0, min_y=0):
    """PosInGrid (:342-353): cvRound((x - minX) * COLS / (maxX - minX)) etc.; returns
    (posX, posY, inside) arrays.  cvRound = round half to even (np.rint)."""
    inv_w = float(FRAME_GRID_COLS) / float(width - min_x)
    inv_h = float(FRAME_GRID_ROWS) / float(height - min_y)
    px = np.rint((np.asarray(x, np.float64) - min_x) * inv_w).astype(np.int64)
    py = np.rint((np.asarray(y, np.float64) - min_y) * inv_h).astype(np.int64)
    inside = (px >= 0) & (px < FRAME_GRID_COLS) & (py >= 0) & (py < FRAME_GRID_ROWS)
    return px, py, inside
