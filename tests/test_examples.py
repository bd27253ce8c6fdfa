"""The reference's example applications (Inception labelling, Johnny CEP) on the runtime."""
import io
import os

import numpy as np
import pytest
import torch
from PIL import Image

from flink_tensorflow_amd.models.zoo.inception import (ImageInputFormat, ImageNormalization, InceptionModel,
                                                        googlenet_like_graph_def)
from flink_tensorflow_amd.runtime import PROCESS_ONCE, StreamExecutionEnvironment
from flink_tensorflow_amd.runtime.cep import CEP, Pattern


def _jpeg(h=64, w=48, seed=0) -> bytes:
    rng = np.random.default_rng(seed)
    buf = io.BytesIO()
    Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(buf, format="JPEG")
    return buf.getvalue()


def test_image_normalization_graph():
    m = ImageNormalization()
    m.open()
    out = m.normalize(_jpeg())
    m.close()
    assert tuple(out.shape) == (1, 224, 224, 3) and out.dtype == torch.float32
    assert -118 <= out.min().item() and out.max().item() <= 139


def test_inception_stream_labels(tmp_path):
    for i in range(3):
        (tmp_path / f"img{i}.jpg").write_bytes(_jpeg(seed=i))
    (tmp_path / "partial.crdownload").write_bytes(b"junk")
    model = InceptionModel(str(tmp_path), image_hw=(64, 48), device="cpu")
    env = StreamExecutionEnvironment.get_execution_environment()
    out = (env.read_file(ImageInputFormat(), str(tmp_path), PROCESS_ONCE)
           .map_with_model(model, lambda rec, m: (rec[0], m.label([rec[1]])[0][0]))
           .execute_and_collect())
    assert sorted(n for n, _ in out) == ["img0.jpg", "img1.jpg", "img2.jpg"]
    for _, (p, label) in out:
        assert 0.0 <= p <= 1.0 and label.startswith("class_")


def test_inception_host_normalized_records(tmp_path):
    (tmp_path / "a.jpeg").write_bytes(_jpeg())
    env = StreamExecutionEnvironment.get_execution_environment()
    out = env.read_file(ImageInputFormat(normalize_on_host=True), str(tmp_path)).execute_and_collect()
    name, tv = out[0]
    assert name == "a.jpeg" and tv.shape() == (1, 224, 224, 3)


def test_googlenet_graph_runs():
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.graph.session import Session

    g = Graph.from_graph_def(googlenet_like_graph_def(num_classes=16, width=0.25))
    y = Session(g).run("output:0", {"input:0": torch.randn(2, 224, 224, 3)})
    assert tuple(y.shape) == (2, 16)
    torch.testing.assert_close(y.sum(-1), torch.ones(2))


def test_johnny_cep():
    """cheeseburger → ladybug → llama within 60 s → AccessGranted; else AccessDenied
    (``EX/inception/johnny.scala:52-62``)."""
    def conf(lbl):
        return lambda v: v[1] == lbl and v[0] >= 0.5

    pattern = (Pattern.begin("first").where(conf("cheeseburger"))
               .followed_by("second").where(conf("ladybug"))
               .followed_by("third").where(conf("llama")).within(60))
    events = [(0.9, "cheeseburger", 0.0), (0.3, "ladybug", 1.0), (0.8, "ladybug", 2.0), (0.7, "cat", 3.0),
              (0.95, "llama", 4.0),                                  # granted (t=0..4)
              (0.9, "cheeseburger", 100.0), (0.9, "ladybug", 110.0),  # times out at 160
              (0.9, "llama", 170.0)]
    env = StreamExecutionEnvironment.get_execution_environment()
    stream = env.from_collection(events).assign_timestamps_and_watermarks(lambda e: e[2])
    out = CEP.pattern(stream, pattern).select(lambda m: ("AccessGranted", m["third"][2]),
                                              lambda partial, ts: ("AccessDenied", ts)).execute_and_collect()
    assert ("AccessGranted", 4.0) in out
    assert ("AccessDenied", 160.0) in out


def test_inception_package_type_aliases():
    """``EX/inception/package.scala:7-30`` aliases: rank / dtype checked at tagging time."""
    import torch

    from flink_tensorflow_amd.models.zoo import inception as I
    from flink_tensorflow_amd.types.tensor import StringTensor

    assert I.as_image_tensor(torch.zeros(2, 224, 224, 3)).shape == (2, 224, 224, 3)
    assert I.as_label_tensor(torch.zeros(2, 1008)).shape == (2, 1008)
    I.ImageFileTensor.check(StringTensor([b"\xff\xd8jpeg"], ()))
    with pytest.raises(TypeError):
        I.as_image_tensor(torch.zeros(224, 224, 3))
    with pytest.raises(TypeError):
        I.as_label_tensor(torch.zeros(2, 1008, dtype=torch.int32))


def test_bert_stream_over_a_savedmodel(tmp_path):
    """examples/bert_stream.py: sentences -> tokenizer -> micro-batched BERT SavedModel ->
    (sentence, label, confidence); every record classified, labels agree with a direct
    (interpreter) call on the same ids."""
    import sys

    import numpy as np

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import bert_stream as bs

    from flink_tensorflow_amd.models import PredictMethod, SavedModelModel
    from flink_tensorflow_amd.models.zoo.bert import BertConfig, HashingTokenizer
    from flink_tensorflow_amd.models.zoo.bert_graph import export_bert_saved_model

    cfg = BertConfig.tiny()
    d = export_bert_saved_model(str(tmp_path / "bert"), cfg, 32, seed=1, mask_from_ids=True)
    env, sink = bs.build_job(d, 40, 8, 32, cfg.vocab_size, delay_ms=1.0, sync=True)
    env.execute("bert-stream")
    out = sorted(sink.results())
    assert len(out) == 40 and all(0.5 <= c <= 1.0 for _, _, c in out)
    tok = HashingTokenizer(cfg.vocab_size, 32)
    m = SavedModelModel(d, device="cpu")
    m.open()
    sents = [s for s, _, _ in out]
    p = m.function("serving_default", PredictMethod(), compile=False).apply(
        {"input_ids": np.stack([tok(s) for s in sents])})["probabilities"]
    assert [lab for _, lab, _ in out] == p.argmax(-1).tolist()
    # default path: SignatureBatchedModel behind the pipelined runner (interpreter on the
    # host), results (label, confidence) in source order
    env, sink = bs.build_job(d, 40, 16, 32, cfg.vocab_size, delay_ms=1.0)
    env.execute("bert-stream-pipelined")
    got = sink.results()
    p = m.function("serving_default", PredictMethod(), compile=False).apply(
        {"input_ids": np.stack([tok(s) for s in bs.sentences(40)])})["probabilities"]
    assert [lab for lab, _ in got] == p.argmax(-1).tolist()
    np.testing.assert_allclose([c for _, c in got], p.max(-1).values.numpy(), rtol=1e-5)
    m.close()


@pytest.mark.parametrize("args", [[], ["--parallelism", "2"], ["--control-stream", "--eval-every", "0.5"]],
                         ids=["generated", "generated-p2", "control-stream"])
def test_widedeep_online_example_cpu(args):
    """examples/widedeep_online.py on the host: the lockstep trainer job trains every click
    record in agreed micro-batch steps — clicks generated in each rank's worker (P = 1, 2)
    or, in the reference's co-process shape, from one coordinator source with a control
    stream of eval ticks — and reports held-out losses."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "examples", "widedeep_online.py"), "--cpu", *args],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["records_trained"] == 2048 and out["steps"] >= 4 and out["eval_losses"]
    assert out["eval_losses"][-1] < 0.6931  # below ln 2, the untrained model's log-loss
