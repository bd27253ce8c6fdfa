"""MNIST-MLP SavedModel (BASELINE CPU plumbing config): export → load → serve in a stream."""
import numpy as np
import pytest
import torch

from flink_tensorflow_amd.io.saver import Saver
from flink_tensorflow_amd.models import RegressionMethod
from flink_tensorflow_amd.models.zoo.mnist import MnistModel, export_mnist_mlp
from flink_tensorflow_amd.runtime import StreamExecutionEnvironment
from flink_tensorflow_amd.types import make_example


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    return export_mnist_mlp(str(tmp_path_factory.mktemp("mnist") / "export"))


def test_export_roundtrip(mnist_dir):
    m = MnistModel(mnist_dir)
    assert sorted(m.metagraph.signature_def) == ["classify_images", "regress_examples", "serving_default"]
    m.open()
    x = torch.rand(5, 784)
    out = m.predict(x)
    torch.testing.assert_close(out["scores"].sum(-1), torch.ones(5))
    classes, scores = m.classify(x)
    assert torch.equal(classes, scores.argmax(-1))
    exs = [make_example(pixels=x[i].tolist()) for i in range(5)]
    p0 = m.function("regress_examples", RegressionMethod()).apply(exs)
    torch.testing.assert_close(p0.reshape(-1), scores[:, 0])
    m.close()


def test_saver_on_exported_model(mnist_dir, tmp_path):
    m = MnistModel(mnist_dir)
    m.open()
    sess = m.session()
    saver = Saver.create(m.metagraph.saver_def)
    before = sess.run("dense/bias:0").clone()
    p = saver.save(sess, str(tmp_path / "ckpt"))
    sess.variables["dense/bias"].fill_(5.0)
    saver.restore(sess, p)
    assert torch.equal(sess.run("dense/bias:0"), before)
    m.close()


@pytest.mark.parametrize("parallelism,batched", [(1, False), (4, True)])
def test_mnist_stream(mnist_dir, parallelism, batched):
    rng = np.random.default_rng(0)
    imgs = rng.random((64, 784), dtype=np.float32)
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(parallelism)
    src = env.from_collection(list(range(64))).rebalance()
    model = MnistModel(mnist_dir)
    if batched:
        out = src.map_with_model_batched(
            model, lambda m, ids: m.classify(torch.from_numpy(imgs[ids]))[0].tolist(), max_batch=16,
            max_delay_ms=1).execute_and_collect()
    else:
        out = src.map_with_model(model, lambda i, m: int(m.classify(torch.from_numpy(imgs[i:i + 1]))[0])) \
            .execute_and_collect()
    ref = MnistModel(mnist_dir)
    ref.open()
    want = ref.classify(torch.from_numpy(imgs))[0].tolist()
    ref.close()
    assert sorted(out) == sorted(want)
