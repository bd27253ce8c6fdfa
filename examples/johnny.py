#!/usr/bin/env python3
""""Johnny" CEP demo — ``EX/inception/johnny.scala:21-80``.

    python examples/johnny.py <model-dir> <images-dir> [--polls N]

Continuously monitors <images-dir> (PROCESS_CONTINUOUSLY, 1 s), labels new images and
grants access when a cheeseburger, a ladybug and a llama (each with confidence >= 0.5)
are seen in that order within 60 seconds; partial sequences time out as AccessDenied.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat, InceptionModel  # noqa: E402
from flink_tensorflow_amd.runtime import PROCESS_CONTINUOUSLY, StreamExecutionEnvironment  # noqa: E402
from flink_tensorflow_amd.runtime.cep import CEP, Pattern  # noqa: E402


def label_is(name, threshold=0.5):
    return lambda v: any(lbl == name and p >= threshold for p, lbl in v[1])


def build_job(env, model, images_dir: str, polls=None, interval_s: float = 1.0, image_hw=(224, 224),
              workers: bool = False):
    """The Johnny pipeline: monitor ``images_dir`` continuously → label each new image with
    ``model`` (``label([img]) -> [[(p, label), ...]]``) → CEP.  The readers run at the
    environment's parallelism and, with ``workers``, are chained with the model operator in
    its worker processes.  Returns the CEP result stream."""
    images = env.read_file(ImageInputFormat(resize_to=image_hw), images_dir, PROCESS_CONTINUOUSLY, interval_s,
                           max_polls=polls)
    labels = images.map_with_model(model, lambda rec, m: (rec[0], m.label([rec[1]])[0]))
    if workers:
        labels = labels.run_in_processes()
    # CEP needs the labels in arrival order on one subtask
    labels = labels.global_() if env.parallelism > 1 else labels
    pattern = (Pattern.begin("first").where(label_is("cheeseburger"))
               .followed_by("second").where(label_is("ladybug"))
               .followed_by("third").where(label_is("llama")).within(60))
    return CEP.pattern(labels, pattern).select(
        lambda m: ("AccessGranted", [m[k][0] for k in ("first", "second", "third")]),
        lambda partial, ts: ("AccessDenied", sorted(partial)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model_dir")
    ap.add_argument("images_dir")
    ap.add_argument("--polls", type=int, default=None, help="stop after N directory polls (default: run forever)")
    a = ap.parse_args()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    build_job(env, InceptionModel(a.model_dir, image_hw=(224, 224)), a.images_dir, a.polls).print()
    env.execute("Johnny")


if __name__ == "__main__":
    main()
