def register(*a, **k):
    pass
