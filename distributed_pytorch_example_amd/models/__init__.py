"""Model zoo: the reference's SimpleNet plus the BASELINE-scope ResNet-50 and GPT-2-small."""
from .simplenet import SimpleNet
from .resnet import ResNet, resnet50, resnet18_like


def get_model(name: str, **kw):
    name = name.lower()
    if name == "simplenet":
        return SimpleNet(**kw)
    if name == "resnet50":
        return resnet50(**kw)
    if name in ("resnet_tiny", "resnet18_like"):
        return resnet18_like(**kw)
    if name in ("gpt2", "gpt2-small", "gpt2_small"):
        from .gpt2 import GPT2, GPT2Config

        return GPT2(GPT2Config(**kw))
    if name in ("gpt2-tiny", "gpt2_tiny"):
        from .gpt2 import GPT2, GPT2Config

        return GPT2(GPT2Config.tiny(**kw))
    raise ValueError(f"unknown model {name!r}")


__all__ = ["SimpleNet", "ResNet", "resnet50", "resnet18_like", "get_model"]
