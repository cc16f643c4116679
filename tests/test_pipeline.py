"""Config-5 pipeline (islpose/pipeline.py): per-frame JSON / feature rows in the
reference's format (extract_features_mp.py:58-108), resume, video sharding over
2 gloo ranks (CPU) and, with -m gpu, the real engine end to end."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from islpose import pipeline


class FakeModel:
    """Stand-in for ISLSignPos.call_batch: a deterministic (candidate, subset, hands)
    per frame that depends on the BGR pixels it receives."""

    def __init__(self):
        self.calls = []

    def call_batch(self, frames_bgr):
        self.calls.append(len(frames_bgr))
        out = []
        for f in frames_bgr:
            v = float(f[0, 0, 0])          # blue channel of pixel (0,0): proves the ::-1 flip
            cand = np.array([[10.0, 20.0, 0.5, 0.0], [v, 30.0, 0.25, 1.0]])
            subset = np.full((1, 27), -1.0)
            subset[0, 0], subset[0, 1], subset[0, -2], subset[0, -1] = 0, 1, 1.5, 2
            hands = [np.array([[0, 0]] + [[5 + i, 6 + i] for i in range(20)], np.int64)]
            out.append((cand, subset, hands))
        return out


def _videos(tmp_path, n_videos=3, T=5):
    base = tmp_path / "data"
    os.makedirs(base / "vids", exist_ok=True)
    rows = []
    for k in range(n_videos):
        fr = np.zeros((T, 8, 10, 3), np.uint8)
        fr[:, 0, 0, 2] = np.arange(T) + 10 * k        # R channel of RGB -> B of BGR
        np.save(base / "vids" / ("v%d.npy" % k), fr)
        rows.append({"Filepath": "vids/v%d.npy" % k, "type": "Adjectives", "expression": "e%d" % k})
    return str(base), rows


def test_frame_json_matches_reference_format():
    cand = np.array([[1.0, 2.0, 0.5, 0.0]])
    subset = np.array([[0.0] + [-1.0] * 24 + [0.5, 1.0]])
    hands = [np.zeros((21, 2), np.int64)]
    ref = json.dumps({'candidate': cand.tolist(), 'subset': subset.tolist(),
                      'all_hand_peaks': [p.tolist() for p in hands]})   # extract_features_mp.py:79-84
    assert pipeline.frame_json(cand, subset, hands) == ref
    # the empty candidate of body.py:183 (shape (0,)) and no hands
    assert pipeline.frame_json(np.array([]), np.zeros((0, 27)), []) == \
        '{"candidate": [], "subset": [], "all_hand_peaks": []}'
    p = pipeline.json_path("/o", "Adjectives", "loud", "MVI_1.MOV", 7)
    assert p == "/o/transforms/Adjectives/loud/MVI_1-original/MVI_1.MOV-7.json"


def test_extract_writes_json_rows_and_resumes(tmp_path):
    base, rows = _videos(tmp_path)
    out = str(tmp_path / "out")
    model = FakeModel()
    feats, ex = pipeline.extract_dataset(rows, pipeline.npy_decoder(base), model, out, batch=2)
    assert len(feats) == 15 and ex.frames_done == 15 and model.calls == [2, 2, 1] * 3
    f = feats[7]                                    # video 1, frame 2
    assert f['frame_no'] == 2 and f['type'] == "Adjectives" and f['expression'] == "e1"
    assert f['candidate'][1][0] == 12.0             # BGR flip: B = RGB's R channel = 2 + 10
    with open(f['filepath']) as fh:
        assert json.load(fh)['candidate'] == f['candidate']
    assert f['bodypose_x_ytupple'] == [(10.0, 20.0), (12.0, 30.0)]
    assert len(f['handpose_peaks'][0]) == 21 and f['handpose_peaks'][1] == []
    # resume: every JSON exists -> nothing recomputed
    model2 = FakeModel()
    feats2, ex2 = pipeline.extract_dataset(rows, pipeline.npy_decoder(base), model2, out, batch=2)
    assert feats2 == [] and ex2.frames_skipped == 15 and model2.calls == []
    os.remove(f['filepath'])
    feats3, _ = pipeline.extract_dataset(rows, pipeline.npy_decoder(base), FakeModel(), out, batch=2)
    assert [r['frame_no'] for r in feats3] == [2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, base, rows, out, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    merged, stats = pipeline.run(rows, pipeline.npy_decoder(base), FakeModel(), out, rank, world, batch=4)
    q.put((rank, stats, None if merged is None else [(m['filepath'], m['frame_no']) for m in merged]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_shard_videos_gloo(tmp_path):
    base, rows = _videos(tmp_path, n_videos=3, T=4)
    out = str(tmp_path / "out")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, base, rows, out, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, stats, merged = q.get(timeout=120)
        res[rank] = (stats, merged)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[0][0]["frames"] == 8 and res[1][0]["frames"] == 4       # videos 0,1 | 2
    merged = res[0][1]
    assert len(merged) == 12 and res[1][1] is None
    assert merged == sorted(merged)
    csvs = [f for f in os.listdir(out) if f.endswith(".csv")]
    assert len(csvs) == 3                                               # one per rank + combined


@pytest.mark.gpu
def test_pipeline_gpu_matches_isl_sign_pos(tmp_path):
    """Real engine (synthetic weights) through the pipeline == ISLSignPos.call per frame."""
    import torch
    from islpose import synth
    from src.body import Body
    from src.hand import Hand
    from src.ISL_Model_parameter import ISLSignPos
    w = lambda k: {n: torch.from_numpy(v) for n, v in synth.synth_weights(k).items()}  # noqa: E731
    isl = ISLSignPos(Body(w(0), "body25").model, Hand(w(2)).model)
    base = tmp_path / "data"
    os.makedirs(base, exist_ok=True)
    frames = synth.synth_frames(3, 240, 320, seed=31)
    np.save(base / "clip.npy", frames)
    rows = [{"Filepath": "clip.npy", "type": "T", "expression": "x"}]
    # export=False: random weights find many people, and the reference's get_handpose
    # export (two hand slots) raises IndexError on a third hand, as it does in the reference
    feats, _ = pipeline.extract_dataset(rows, pipeline.npy_decoder(str(base)), isl, str(tmp_path / "o"), batch=2,
                                        export=False)
    assert len(feats) == 3
    for i, f in enumerate(feats):
        ref = isl.call(np.ascontiguousarray(frames[i][:, :, ::-1]))
        with open(f['filepath']) as fh:
            assert fh.read() == pipeline.frame_json(*ref)


@pytest.mark.gpu
def test_pipeline_overlap_equals_sequential(tmp_path):
    """The overlapped pipeline (prefetch thread + pinned ring + copy stream, GPU flip,
    writer thread) writes what the sequential loop writes, over several videos and
    ragged batches (5 frames, batch 2), and resumes the same way."""
    base, rows = _videos(tmp_path, n_videos=3, T=5)
    outs = {}
    for ov in (False, True):
        out = str(tmp_path / ("out%d" % ov))
        model = FakeModel()
        feats, ex = pipeline.extract_dataset(rows, pipeline.npy_decoder(base), model, out, batch=2, overlap=ov)
        assert ex.frames_done == 15 and model.calls == [2, 2, 1] * 3
        outs[ov] = feats
        texts = []
        for f in feats:
            with open(f['filepath']) as fh:
                texts.append(fh.read())
        outs[ov] = ([{k: v for k, v in f.items() if k != 'filepath'} for f in feats], texts)
    assert outs[True] == outs[False]
    # resume under overlap: nothing recomputed
    model = FakeModel()
    feats, ex = pipeline.extract_dataset(rows, pipeline.npy_decoder(base), model, str(tmp_path / "out1"),
                                         batch=2, overlap=True)
    assert feats == [] and ex.frames_skipped == 15 and model.calls == []
