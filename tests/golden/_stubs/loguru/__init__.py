class _Logger:
    def __getattr__(self, name):
        return lambda *a, **k: None


logger = _Logger()
