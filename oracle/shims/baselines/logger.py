def log(*a, **k):
    pass
