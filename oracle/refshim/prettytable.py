"""import-time stub (test-only)"""


class PrettyTable(object):
    def __init__(self, *a, **k):
        pass

    def add_row(self, *a, **k):
        pass
