class RecordConstructorArgs:
    def __init__(self, **kwargs):
        self._saved_kwargs = kwargs
