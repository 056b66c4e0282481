"""No-op wandb stand-in (fixture generation only)."""
run = None


def init(*a, **k):
    return None


def log(*a, **k):
    pass


def save(*a, **k):
    pass
