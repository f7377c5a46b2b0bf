class ParameterError(Exception):
    pass
