"""Config 5 pipeline: videos -> body + hand keypoints -> per-frame JSON, one process per GPU.

The MI355X counterpart of the reference's feature extractor
(extract_features_mp.py):

* per-frame output = the reference's JSON, byte for byte: ``json.dump`` of
  ``{'candidate', 'subset', 'all_hand_peaks'}`` via ``.tolist()``
  (extract_features_mp.py:79-84), at the same path
  ``<out>/transforms/<type>/<expression>/<stem>-original/<filename>-<idx>.json``
  (:62-66, :77);
* per-frame feature rows = the reference's ``features`` dict (:94-108), written
  as one CSV per rank (``saveFeaturesDict``, :58-63) and gathered on rank 0
  (the mp.Queue of :204-231, here a host-side gather of a few KB per frame);
* resume: frames whose JSON already exists are skipped (extract_features.py:97-101);
* the frame fed to the model is ``frame[:, :, ::-1]`` (RGB video -> BGR, :124).

What differs, MI355X-first: frames go to the GPU in batches (``ISLSignPos.call_batch``:
one body launch sequence per batch instead of per frame), every rank pins its
own device (the reference ran every worker on cuda:0, body.py:32), and videos
are sharded across ranks with no collective on the data path.

Video decoding: ``pims``/``torchvision.io`` are absent from this image, so the
decoder is a parameter; ``npy_decoder`` reads uint8 [T,H,W,3] RGB arrays and
``synthetic_decoder`` makes seeded frames (benchmarks).
"""
from __future__ import annotations

import csv
import datetime
import json
import os
import time

import numpy as np

from .parallel import gather_to_rank0, shard_bounds


def frame_json(candidate, subset, all_hand_peaks) -> str:
    """The reference's per-frame JSON text (extract_features_mp.py:79-84)."""
    return json.dumps({
        'candidate': np.asarray(candidate).tolist(),
        'subset': np.asarray(subset).tolist(),
        'all_hand_peaks': [np.asarray(p).tolist() for p in all_hand_peaks],
    })


def json_path(out_base: str, label_type: str, expression: str, filename: str, idx: int,
              transform: str = "original") -> str:
    """extract_features_mp.py:62-66,77: <base>/transforms/<type>/<expr>/<stem>-<transform>/<filename>-<idx>.json"""
    d = os.path.join(out_base, "transforms", label_type, expression, "%s-%s" % (filename.split('.')[0], transform))
    return os.path.join(d, "%s-%d.json" % (filename, idx))


def feature_row(path: str, idx: int, label_type: str, expression: str, feature, transform: str = "original",
                export: bool = True):
    """The reference's per-frame feature dict (extract_features_mp.py:94-108).  Its
    get_handpose export has two hand slots, so a frame with more than two hands
    raises IndexError there, as in the reference; export=False leaves the four
    export columns out."""
    candidate, subset, hands = feature
    row = {
        'transform': transform, 'filepath': path, 'frame_no': idx, 'type': label_type,
        'expression': expression, 'candidate': np.asarray(candidate).tolist(),
        'subset': np.asarray(subset).tolist(), 'all_hand_peaks': [np.asarray(p).tolist() for p in hands],
    }
    if export:
        from src.util import get_bodypose, get_handpose
        body_xy, body_sticks = get_bodypose(candidate, subset, 'body25')
        hand_edges, hand_peaks = get_handpose(hands)
        row.update({'bodypose_x_ytupple': body_xy, 'bodypose_x_y_sticks': body_sticks,
                    'handpose_edges': hand_edges, 'handpose_peaks': hand_peaks})
    return row


def npy_decoder(dataset_base: str):
    """Filepath (relative to dataset_base) of a .npy uint8 [T,H,W,3] RGB video -> frames."""
    def decode(filepath):
        return np.load(os.path.join(dataset_base, filepath), mmap_mode="r")
    return decode


def synthetic_decoder(n_frames: int, h: int, w: int):
    """Seeded synthetic RGB frames; the video's frames depend only on its Filepath."""
    import zlib
    from .synth import synth_frames

    def decode(filepath):
        return synth_frames(n_frames, h, w, seed=zlib.crc32(filepath.encode()) & 0x7FFFFFFF)
    return decode


class KeypointExtractor:
    """Runs `model.call_batch(bgr_frames) -> [(candidate, subset, all_hand_peaks)]` over
    videos in batches and writes the reference's per-frame outputs."""

    def __init__(self, model, out_base: str, batch: int = 64, resume: bool = True, write_json: bool = True,
                 export: bool = True):
        self.model = model
        self.export = export
        self.out_base = out_base
        self.batch = batch
        self.resume = resume
        self.write_json = write_json
        self.frames_done = 0
        self.frames_skipped = 0

    def run_video(self, filename: str, frames, label_type: str, expression: str):
        rows = []
        todo = []
        for idx in range(len(frames)):
            p = json_path(self.out_base, label_type, expression, filename, idx)
            if self.resume and os.path.exists(p):
                self.frames_skipped += 1
                continue
            todo.append(idx)
        for s in range(0, len(todo), self.batch):
            ids = todo[s:s + self.batch]
            # model(frame[:, :, ::-1]): the reference feeds BGR (extract_features_mp.py:124)
            bgr = np.ascontiguousarray(np.stack([np.asarray(frames[i]) for i in ids])[..., ::-1])
            feats = self.model.call_batch(bgr)
            for idx, feat in zip(ids, feats):
                p = json_path(self.out_base, label_type, expression, filename, idx)
                if self.write_json:
                    os.makedirs(os.path.dirname(p), exist_ok=True)
                    with open(p, "w") as f:
                        f.write(frame_json(*feat))
                rows.append(feature_row(p, idx, label_type, expression, feat, export=self.export))
            self.frames_done += len(ids)
        return rows


def extract_dataset(rows, decode, model, out_base: str, rank: int = 0, world: int = 1, batch: int = 64,
                    resume: bool = True, write_json: bool = True, export: bool = True):
    """rows: [{'Filepath', 'type', 'expression'}] (the dataset CSV of extract_features_mp.py:187).
    Videos are sharded contiguously across ranks; returns (this rank's feature rows, extractor)."""
    start, end = shard_bounds(len(rows), rank, world)
    ex = KeypointExtractor(model, out_base, batch=batch, resume=resume, write_json=write_json, export=export)
    out = []
    for r in rows[start:end]:
        fp = r['Filepath']
        out.extend(ex.run_video(fp.split('/')[-1], decode(fp), r['type'], r['expression']))
    return out, ex


def save_features_csv(features, path: str):
    """saveFeaturesDict (extract_features_mp.py:58-63): one row per frame."""
    import pandas as pd
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    pd.DataFrame(features).to_csv(path, index=False)
    return path


def read_dataset_csv(path: str):
    with open(path, newline="") as f:
        return [dict(r) for r in csv.DictReader(f)]


def run(rows, decode, model, out_base: str, rank: int, world: int, batch: int = 64, resume: bool = True,
        write_json: bool = True, group=None, export: bool = True):
    """One rank's share + the host-side gather; rank 0 writes the combined CSV like the
    reference's __main__ (extract_features_mp.py:225-239). Returns (rows on rank 0 or None, stats)."""
    t0 = time.time()
    feats, ex = extract_dataset(rows, decode, model, out_base, rank, world, batch, resume, write_json, export)
    dt = time.time() - t0
    stamp = datetime.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    save_features_csv(feats, os.path.join(out_base, "output_%d_exectime-%.4f_%s.csv" % (rank, dt, stamp)))
    tagged = [((r['filepath'], r['frame_no']), r) for r in feats]
    merged = gather_to_rank0(tagged, rank, world, group=group)
    stats = {"rank": rank, "frames": ex.frames_done, "skipped": ex.frames_skipped, "seconds": dt}
    if rank == 0:
        save_features_csv(merged, os.path.join(out_base, "output_%s_exectime-%.4f.csv" % (stamp, time.time() - t0)))
    return merged, stats
