from .fused import SGD, Adam, AdamW

__all__ = ["SGD", "Adam", "AdamW"]


def build_optimizer(name: str, params, lr: float, weight_decay: float = 0.0, momentum: float = 0.9):
    name = name.lower()
    if name == "adam":
        return Adam(params, lr=lr, weight_decay=weight_decay)
    if name == "adamw":
        return AdamW(params, lr=lr, weight_decay=weight_decay)
    if name == "sgd":
        return SGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay)
    raise ValueError(f"unknown optimizer {name!r}")
