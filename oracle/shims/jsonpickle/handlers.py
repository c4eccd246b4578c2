class BaseHandler:
    def __init__(self, context=None):
        self.context = context


def register(cls, handler=None, base=False):
    def deco(h):
        return h
    return deco if handler is None else handler
