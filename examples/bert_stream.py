#!/usr/bin/env python3
"""BERT text-classification stream over a TF SavedModel, on the DataStream runtime.

    python examples/bert_stream.py [--export-dir DIR] [--records N] [--batch 64] [--tiny]

sentence source -> tokenize (HashingTokenizer) -> map_with_model_batched(SavedModelModel):
each micro-batch runs ``model.function("serving_default", PredictMethod())`` — on a GPU the
signature is compiled once per batch bucket (fused QKV GEMM + flash attention + fused
LayerNorm / GELU epilogues, hipGraph), on the CPU it runs on the interpreter — -> sink of
(sentence, label, confidence).  Without ``--export-dir`` a random-init BERT SavedModel is
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

from flink_tensorflow_amd.models import PredictMethod, SavedModelModel  # noqa: E402
from flink_tensorflow_amd.models.zoo.bert import BertConfig, HashingTokenizer  # noqa: E402
from flink_tensorflow_amd.models.zoo.bert_graph import export_bert_saved_model  # noqa: E402
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment  # noqa: E402

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


def build_job(export_dir, n, batch, seq, vocab, delay_ms=5.0):
    tok = HashingTokenizer(vocab, seq)
    env = StreamExecutionEnvironment.get_execution_environment()
    sink = env.from_collection(sentences(n)).map(lambda s: (s, tok(s))) \
        .map_with_model_batched(SavedModelModel(export_dir), classify, max_batch=batch, max_delay_ms=delay_ms,
                                name="bert").collect_into()
    return env, sink


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--export-dir", default=None)
    ap.add_argument("--records", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--tiny", action="store_true")
    a = ap.parse_args()
    cfg = BertConfig.tiny() if a.tiny else BertConfig.base()
    d = a.export_dir
    if d is None or not os.path.exists(os.path.join(d, "saved_model.pb")):
        d = d or os.path.join(tempfile.mkdtemp(), "bert")
        export_bert_saved_model(d, cfg, a.seq, seed=0, mask_from_ids=True)
    env, sink = build_job(d, a.records, a.batch, a.seq, cfg.vocab_size)
    t0 = time.time()
    res = env.execute("bert-stream")
    el = time.time() - t0
    out = sink.results()
    m = [v for k, v in res.metrics.items() if k.startswith("bert")][0]
    print(json.dumps({"records": len(out), "seconds": round(el, 3), "records_per_s": round(len(out) / el, 1),
                      "latency_s": m["histograms"].get("latency_s"), "sample": out[:2]}))


if __name__ == "__main__":
    main()
