#!/usr/bin/env python3
"""BERT text-classification stream over a TF SavedModel, on the DataStream runtime.

    python examples/bert_stream.py [--export-dir DIR] [--records N] [--batch 256] [--tiny] [--sync]

sentence source -> tokenize (HashingTokenizer) -> map_with_model_batched(model) -> sink.
Default: ``SignatureBatchedModel(export_dir)`` — the ``serving_default`` signature compiled
per batch bucket and compute lane (fused QKV GEMM + flash attention + fused LayerNorm /
GELU epilogues, hipGraph) behind the pipelined pinned-H2D runner; results are
(label, confidence).  ``--sync``: a batch function calling
``SavedModelModel.function("serving_default", PredictMethod())`` per micro-batch (one call
at a time); results are (sentence, label, confidence).  On a CPU both run on the
interpreter.  Without ``--export-dir`` a random-init BERT SavedModel is
exported first (there is no network to fetch a trained one); with ``--tiny`` a 2-layer
model, so the example runs in seconds on a laptop CPU.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.models import PredictMethod, SavedModelModel, SignatureBatchedModel  # noqa: E402
from flink_tensorflow_amd.models.zoo.bert import BertConfig, HashingTokenizer  # noqa: E402
from flink_tensorflow_amd.models.zoo.bert_graph import export_bert_saved_model  # noqa: E402
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment  # noqa: E402
from flink_tensorflow_amd.runtime.sources import ThroughputSink  # noqa: E402

WORDS = ("the stream of records flows through the engine while the model labels every sentence it sees "
         "fast gpu kernels make inference cheap and latency low for every tenant of the cluster").split()


def sentences(n, seed=0):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, int(rng.integers(4, 24)))) for _ in range(n)]


def classify(model, batch):
    """``batch``: [(sentence, ids)] -> [(sentence, label, confidence)]."""
    ids = np.stack([b[1] for b in batch])
    out = model.function("serving_default", PredictMethod()).apply({"input_ids": ids})
    p = out["probabilities"].float().cpu().numpy()
    return [(s, int(p[i].argmax()), float(p[i].max())) for i, (s, _) in enumerate(batch)]


def label(result):
    p = result["probabilities"]
    return int(p.argmax()), float(p.max())


def build_job(export_dir, n, batch, seq, vocab, delay_ms=5.0, sync=False, lanes=2, sink=None):
    tok = HashingTokenizer(vocab, seq)
    env = StreamExecutionEnvironment.get_execution_environment()
    src = env.from_collection(sentences(n))
    if sync:
        out = src.map(lambda s: (s, tok(s))).map_with_model_batched(
            SavedModelModel(export_dir), classify, max_batch=batch, max_delay_ms=delay_ms, name="bert")
    else:
        model = SignatureBatchedModel(export_dir, buckets=sorted({min(64, batch), batch}), lanes=lanes)
        out = src.map(tok).map_with_model_batched(model, None, max_batch=batch, max_delay_ms=delay_ms,
                                                  name="bert").map(label)
    if sink is not None:
        out.add_sink(sink)
        return env, sink
    return env, out.collect_into()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--export-dir", default=None)
    ap.add_argument("--records", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--sync", action="store_true", help="one ModelFunction call per micro-batch")
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--steady", action="store_true",
                    help="count results in a ThroughputSink and report the steady-state rate")
    a = ap.parse_args()
    cfg = BertConfig.tiny() if a.tiny else BertConfig.base()
    d = a.export_dir
    if d is None or not os.path.exists(os.path.join(d, "saved_model.pb")):
        d = d or os.path.join(tempfile.mkdtemp(), "bert")
        export_bert_saved_model(d, cfg, a.seq, seed=0, mask_from_ids=True)
    sink = ThroughputSink() if a.steady else None
    env, sink = build_job(d, a.records, a.batch, a.seq, cfg.vocab_size, sync=a.sync, lanes=a.lanes, sink=sink)
    t0 = time.time()
    res = env.execute("bert-stream")
    el = time.time() - t0
    m = [v for k, v in res.metrics.items() if k.startswith("bert")][0]
    if a.steady:  # skip the first fifth (compile, capture, pipeline fill)
        extra = {"steady_records_per_s": round(sink.rate(0.2) or 0.0, 1)}
        n = a.records
    else:
        out = sink.results()
        extra = {"sample": out[:2]}
        n = len(out)
    print(json.dumps({"records": n, "path": "sync" if a.sync else "pipelined", "seconds": round(el, 3),
                      "records_per_s": round(n / el, 1), "latency_s": m["histograms"].get("latency_s"), **extra}))


if __name__ == "__main__":
    main()
