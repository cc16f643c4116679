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


class _Prefetch:
    """Host -> device staging ahead of the compute (async H2D).

    A background thread reads each batch's frames (the "decode": a slice of an
    mmap-ed / in-memory uint8 RGB video) into one of a ring of pinned host buffers
    and issues the H2D copy on its own HIP stream; the consumer makes its stream wait
    on the copy's event.  So while the GPU runs batch i, batch i+1 is read and
    uploaded.  The ring has depth + 1 slots: a slot is refilled only after the event
    of its previous copy has completed."""

    def __init__(self, jobs, device: int, depth: int = 2):
        import queue
        import threading
        import torch
        self.torch = torch
        self.device = device
        self.q = queue.Queue(maxsize=depth)
        self.slots = [None] * (depth + 1)
        self.events = [None] * (depth + 1)
        self.stream = torch.cuda.Stream(device=device)
        self.error = None
        self.thread = threading.Thread(target=self._run, args=(jobs,), daemon=True)
        self.thread.start()

    def _run(self, jobs):
        torch = self.torch
        try:
            torch.cuda.set_device(self.device)
            for k, (meta, frames) in enumerate(jobs):
                i = k % len(self.slots)
                if self.events[i] is not None:
                    self.events[i].synchronize()          # the slot's previous upload is done
                n, shape = len(frames), tuple(frames.shape[1:])
                buf = self.slots[i]
                if buf is None or buf.shape[0] < n or tuple(buf.shape[1:]) != shape:
                    buf = self.slots[i] = torch.empty((n,) + shape, dtype=torch.uint8, pin_memory=True)
                np.copyto(buf[:n].numpy(), np.asarray(frames))
                with torch.cuda.stream(self.stream):
                    dev = torch.empty((n,) + shape, dtype=torch.uint8, device="cuda:%d" % self.device)
                    dev.copy_(buf[:n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.events[i] = ev
                self.q.put((meta, dev, ev))
        except BaseException as e:  # surfaced to the consumer
            self.error = e
        self.q.put(None)

    def __iter__(self):
        torch = self.torch
        cur = torch.cuda.current_stream(self.device)
        while True:
            item = self.q.get()
            if item is None:
                if self.error is not None:
                    raise self.error
                return
            meta, dev, ev = item
            cur.wait_event(ev)
            dev.record_stream(cur)      # the allocator must not recycle it before the compute ran
            yield meta, dev


class _Writer:
    """JSON files and feature rows on a background thread, off the GPU's critical path."""

    def __init__(self, fn):
        import queue
        import threading
        self.q = queue.Queue(maxsize=4)
        self.fn = fn
        self.error = None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            if self.error is None:
                try:
                    self.fn(*item)
                except BaseException as e:
                    self.error = e

    def put(self, *item):
        if self.error is not None:
            raise self.error
        self.q.put(item)

    def close(self):
        self.q.put(None)
        self.thread.join()
        if self.error is not None:
            raise self.error


class KeypointExtractor:
    """Runs `model.call_batch(bgr_frames) -> [(candidate, subset, all_hand_peaks)]` over
    videos in batches and writes the reference's per-frame outputs.

    overlap=True (the default when a GPU is visible and the model takes device frames:
    it has call_batches or accepts_device_frames) pipelines the host work around
    the GPU: frames are read and uploaded one batch ahead (_Prefetch, pinned buffers +
    a copy stream), the RGB -> BGR flip of extract_features_mp.py:124 runs on the GPU,
    and the JSON / feature-row writing runs on a writer thread.  The outputs are the
    same as with overlap=False (the sequential loop: host flip, synchronous upload,
    inline writes)."""

    def __init__(self, model, out_base: str, batch: int = 64, resume: bool = True, write_json: bool = True,
                 export: bool = True, overlap=None):
        self.model = model
        self.export = export
        self.out_base = out_base
        self.batch = batch
        self.resume = resume
        self.write_json = write_json
        self.overlap = overlap
        self.frames_done = 0
        self.frames_skipped = 0

    def _todo(self, filename, frames, label_type, expression):
        todo = []
        for idx in range(len(frames)):
            p = json_path(self.out_base, label_type, expression, filename, idx)
            if self.resume and os.path.exists(p):
                self.frames_skipped += 1
                continue
            todo.append(idx)
        return todo

    def _write(self, rows, filename, label_type, expression, ids, feats):
        for idx, feat in zip(ids, feats):
            p = json_path(self.out_base, label_type, expression, filename, idx)
            if self.write_json:
                os.makedirs(os.path.dirname(p), exist_ok=True)
                with open(p, "w") as f:
                    f.write(frame_json(*feat))
            rows.append(feature_row(p, idx, label_type, expression, feat, export=self.export))

    def _batches(self, videos):
        """videos: iterable of (filename, frames, label_type, expression) -> per batch
        ((rows list, filename, label_type, expression, ids), frames of the batch)."""
        for filename, frames, label_type, expression, rows in videos:
            if callable(frames):
                frames = frames()                             # decode lazily (on the prefetch thread)
            todo = self._todo(filename, frames, label_type, expression)
            for s in range(0, len(todo), self.batch):
                ids = todo[s:s + self.batch]
                if ids == list(range(ids[0], ids[-1] + 1)) and hasattr(frames, "shape"):
                    sel = frames[ids[0]:ids[-1] + 1]          # contiguous: a view (mmap / array slice)
                else:
                    sel = np.stack([np.asarray(frames[i]) for i in ids])
                yield (rows, filename, label_type, expression, ids), sel

    def run_videos(self, videos):
        """videos: list of (filename, frames, label_type, expression), frames an array-like
        [T, H, W, 3] uint8 RGB or a callable returning one; returns one list of feature
        rows per video, in order."""
        import torch
        out = [[] for _ in videos]
        vids = [(f, fr, lt, ex, out[k]) for k, (f, fr, lt, ex) in enumerate(videos)]
        # the overlapped path hands the model GPU tensors: by default only models that
        # declare it (ISLSignPos: call_batches / accepts_device_frames) get it; any other
        # model keeps numpy BGR batches
        device_ok = hasattr(self.model, "call_batches") or getattr(self.model, "accepts_device_frames", False)
        overlap = (torch.cuda.is_available() and device_ok) if self.overlap is None else self.overlap
        if not overlap:
            for (rows, filename, lt, ex, ids), sel in self._batches(vids):
                # model(frame[:, :, ::-1]): the reference feeds BGR (extract_features_mp.py:124)
                bgr = np.ascontiguousarray(np.asarray(sel)[..., ::-1])
                self._write(rows, filename, lt, ex, ids, self.model.call_batch(bgr))
                self.frames_done += len(ids)
            return out
        dev = getattr(self.model, "_device", None)
        dev = torch.cuda.current_device() if dev is None else dev
        writer = _Writer(self._write)

        def bgr_batches():
            for meta, rgb in _Prefetch(self._batches(vids), dev):
                yield meta, rgb.flip(-1)                      # extract_features_mp.py:124, on the GPU

        # models with the pipelined form (ISLSignPos.call_batches) overlap the body of
        # batch k with the hands of batch k-1 on the GPU
        batches = getattr(self.model, "call_batches", None)
        if batches is None:
            batches = lambda it: ((meta, self.model.call_batch(bgr)) for meta, bgr in it)  # noqa: E731
        try:
            for (rows, filename, lt, ex, ids), feats in batches(bgr_batches()):
                writer.put(rows, filename, lt, ex, ids, feats)
                self.frames_done += len(ids)
        finally:
            writer.close()
        return out

    def run_video(self, filename: str, frames, label_type: str, expression: str):
        return self.run_videos([(filename, frames, label_type, expression)])[0]


def extract_dataset(rows, decode, model, out_base: str, rank: int = 0, world: int = 1, batch: int = 64,
                    resume: bool = True, write_json: bool = True, export: bool = True, overlap=None):
    """rows: [{'Filepath', 'type', 'expression'}] (the dataset CSV of extract_features_mp.py:187).
    Videos are sharded contiguously across ranks; returns (this rank's feature rows, extractor)."""
    start, end = shard_bounds(len(rows), rank, world)
    ex = KeypointExtractor(model, out_base, batch=batch, resume=resume, write_json=write_json, export=export,
                           overlap=overlap)
    videos = [(r['Filepath'].split('/')[-1], (lambda fp=r['Filepath']: decode(fp)), r['type'], r['expression'])
              for r in rows[start:end]]
    out = []
    for v in ex.run_videos(videos):
        out.extend(v)
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
        write_json: bool = True, group=None, export: bool = True, overlap=None):
    """One rank's share + the host-side gather; rank 0 writes the combined CSV like the
    reference's __main__ (extract_features_mp.py:225-239). Returns (rows on rank 0 or None, stats)."""
    t0 = time.time()
    feats, ex = extract_dataset(rows, decode, model, out_base, rank, world, batch, resume, write_json, export,
                                overlap)
    dt = time.time() - t0
    stamp = datetime.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    save_features_csv(feats, os.path.join(out_base, "output_%d_exectime-%.4f_%s.csv" % (rank, dt, stamp)))
    tagged = [((r['filepath'], r['frame_no']), r) for r in feats]
    merged = gather_to_rank0(tagged, rank, world, group=group)
    stats = {"rank": rank, "frames": ex.frames_done, "skipped": ex.frames_skipped, "seconds": dt}
    if rank == 0:
        save_features_csv(merged, os.path.join(out_base, "output_%s_exectime-%.4f.csv" % (stamp, time.time() - t0)))
    return merged, stats
