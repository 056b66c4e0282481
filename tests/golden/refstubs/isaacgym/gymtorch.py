"""Zero-copy wrap/unwrap stand-ins: the fake gym hands out torch tensors directly."""


def wrap_tensor(t):
    return t


def unwrap_tensor(t):
    return t
