#!/usr/bin/env python3
"""Inception image labelling stream — ``EX/inception/inception.scala:17-53``.

    python examples/inception.py <model-dir> <images-dir> [--gpu-batched]

Reads every ``*.jpg``/``*.jpeg`` under <images-dir> once (PROCESS_ONCE, 1 s monitor
interval), labels it with the Inception graph in <model-dir>
(``tensorflow_inception_graph.pb`` + ``imagenet_comp_graph_label_strings.txt``; a
random-init GoogLeNet-shaped graph is synthesized when the files are absent) and prints
``(file, (probability, label))``.  ``--gpu-batched`` stages records into GPU micro-batches
(fused resize/normalize, MFMA convs, fused top-k) instead of per-record calls.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat, InceptionModel  # noqa: E402
from flink_tensorflow_amd.runtime import PROCESS_ONCE, StreamExecutionEnvironment  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model_dir")
    ap.add_argument("images_dir")
    ap.add_argument("--gpu-batched", action="store_true")
    a = ap.parse_args()
    env = StreamExecutionEnvironment.get_execution_environment().set_parallelism(1)
    images = env.read_file(ImageInputFormat(resize_to=(224, 224)), a.images_dir, PROCESS_ONCE, 1.0)
    model = InceptionModel(a.model_dir, image_hw=(224, 224))
    if a.gpu_batched:
        names = images.map(lambda r: r)  # keep (name, image)
        labelled = names.map_with_model_batched(
            model, lambda m, recs: [(n, lbl[0]) for (n, _), lbl in zip(recs, m.label([img for _, img in recs]))],
            max_batch=64, max_delay_ms=20)
    else:
        labelled = images.map_with_model(model, lambda rec, m: (rec[0], m.label([rec[1]])[0][0]))
    labelled.print()
    env.execute("Inception")


if __name__ == "__main__":
    main()
