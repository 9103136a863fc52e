"""Exception hierarchy of the reference (jwave/exceptions/): JWaveException is
the checked base (JWaveException.java:32), JWaveFailure marks invalid input
(JWaveFailure.java:32), JWaveError marks internal/runtime errors
(JWaveError.java:32).  Native device failures surface as JWaveError."""


class JWaveException(Exception):
    def __init__(self, message=""):
        super().__init__(message)
        self.message = message

    def getMessage(self):  # noqa: N802 (reference name)
        return self.message


class JWaveFailure(JWaveException):
    pass


class JWaveError(JWaveException):
    pass
