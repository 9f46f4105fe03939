"""transformers integration -- the equivalent of the reference README recipe that
patches ``transformers/integrations/bitsandbytes.py::_replace_with_bnb_linear``
(README.md:52-86) to build ``Linear4bit`` instead of ``bnb.nn.Linear4bit``.

Installed transformers (5.x) only routes ``load_in_4bit`` through bitsandbytes,
which does not exist on ROCm here, so the replacement is done explicitly on an
already-built model: every ``nn.Linear`` (except ``modules_to_not_convert``,
``lm_head`` by default as in transformers) becomes a ``Linear4bit`` and its
weight is quantised on the GPU.
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch
import torch.nn as nn

from .core import Params4bit
from .modules import Linear4bit


def _cfg(quantization_config, name, default):
    return getattr(quantization_config, name, default) if quantization_config is not None else default


def replace_with_bnb_linear(model: nn.Module, modules_to_not_convert: Optional[Iterable[str]] = None,
                            quantization_config=None, quant_type: Optional[str] = None,
                            compress_statistics: Optional[bool] = None, compute_dtype=None,
                            device=None) -> nn.Module:
    """Replace nn.Linear modules with Linear4bit (same kwargs the README recipe passes:
    compute dtype, compress_statistics=bnb_4bit_use_double_quant, quant_type,
    quant_storage) and quantise their weights on `device` (default: the weight's
    device, which must be a GPU)."""
    skip = set(modules_to_not_convert or ["lm_head"])
    qt = quant_type or _cfg(quantization_config, "bnb_4bit_quant_type", "nf4")
    cs = compress_statistics if compress_statistics is not None else \
        _cfg(quantization_config, "bnb_4bit_use_double_quant", True)
    cd = compute_dtype if compute_dtype is not None else _cfg(quantization_config, "bnb_4bit_compute_dtype", None)
    qstorage = _cfg(quantization_config, "bnb_4bit_quant_storage", torch.uint8)

    def visit(parent: nn.Module, prefix: str):
        for name, child in list(parent.named_children()):
            full = f"{prefix}.{name}" if prefix else name
            if isinstance(child, nn.Linear) and not isinstance(child, Linear4bit) and \
                    name not in skip and full not in skip:
                dev = torch.device(device) if device is not None else child.weight.device
                new = Linear4bit(child.in_features, child.out_features, child.bias is not None, cd,
                                 compress_statistics=cs, quant_type=qt, quant_storage=qstorage, device="meta")
                new.weight = Params4bit(child.weight.data, requires_grad=False, quant_type=qt,
                                        quant_storage=qstorage, module=new, compress_statistics=cs).to(dev)
                if child.bias is not None:
                    new.bias = nn.Parameter(child.bias.data.to(dev), requires_grad=False)
                parent._modules[name] = new
                del child
            else:
                visit(child, full)

    visit(model, "")
    return model


# the name used by transformers (README.md:67)
_replace_with_bnb_linear = replace_with_bnb_linear
