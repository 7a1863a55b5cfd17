"""Record the parameter and buffer layouts of the reference models BASELINE.json names.

Run in the build container only (the reference tree does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference python3 tests/golden/make_layouts.py

Writes ``tests/golden/layouts.json``: for each model, the ``named_parameters()`` and
``named_buffers()`` names, shapes and dtypes, in module order (the order fedavg.py:24 zips
parameters in).  Data only: no reference source is copied.

* google_speech ResNet-34 and CIFAR-10 ResNet-8 are built by the reference's own
  ``accdfl.core.models.create_model`` (accdfl/core/models/__init__.py:19-51), which imports
  here with torch alone.
* GNLeNet (cifar10 default) and the FEMNIST CNN need ``torchvision`` /
  ``dataclasses_json`` at import, which this container lacks; their layouts are read
  from the source text (accdfl/core/models/cifar10.py:101, accdfl/core/models/femnist.py:45-61:
  conv1 1->32 k5, conv2 32->64 k5, fc1 3136->512, fc2 512->62) and marked ``from_source``.
"""
from __future__ import annotations

import json
import os

from accdfl.core.models import create_model  # the reference, via PYTHONPATH

HERE = os.path.dirname(os.path.abspath(__file__))


def layout(model):
    return {
        "params": [[n, list(p.shape), str(p.dtype).replace("torch.", "")] for n, p in model.named_parameters()],
        "buffers": [[n, list(b.shape), str(b.dtype).replace("torch.", "")] for n, b in model.named_buffers()],
        "from": "create_model",
    }


def main():
    out = {
        "google_speech_resnet34": layout(create_model("google_speech")),
        "cifar10_resnet8": layout(create_model("cifar10", architecture="resnet8")),
        "femnist_cnn": {
            "params": [["conv1.weight", [32, 1, 5, 5], "float32"], ["conv1.bias", [32], "float32"],
                       ["conv2.weight", [64, 32, 5, 5], "float32"], ["conv2.bias", [64], "float32"],
                       ["fc1.weight", [512, 3136], "float32"], ["fc1.bias", [512], "float32"],
                       ["fc2.weight", [62, 512], "float32"], ["fc2.bias", [62], "float32"]],
            "buffers": [], "from": "from_source accdfl/core/models/femnist.py:45-61",
        },
    }
    for name, lay in out.items():
        lay["n_params"] = sum(int(__import__("math").prod(s)) for _, s, _ in lay["params"])
        lay["n_buffer_elems"] = sum(int(__import__("math").prod(s)) for _, s, _ in lay["buffers"])
        print(name, len(lay["params"]), "tensors", lay["n_params"], "params", len(lay["buffers"]), "buffers")
    with open(os.path.join(HERE, "layouts.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
