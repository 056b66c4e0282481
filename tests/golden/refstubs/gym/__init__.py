"""Stand-in for OpenAI gym's Env/Wrapper/spaces (fixture generation only)."""


class Env:
    pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)


class _Spaces:
    class Box:
        def __init__(self, *a, **k):
            pass


spaces = _Spaces()
