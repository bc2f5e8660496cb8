"""No-op stand-in for OpenCV (absent in this image); golden-vector generation only."""


def imshow(*_a, **_k):
    return None


def waitKey(*_a, **_k):
    return -1


def destroyAllWindows(*_a, **_k):
    return None


def namedWindow(*_a, **_k):
    return None
