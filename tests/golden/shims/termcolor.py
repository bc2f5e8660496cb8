"""No-op stand-in for `termcolor` (absent in this image).

Used ONLY by tests/golden/make_golden.py so the read-only reference at
/root/reference can be imported to generate golden vectors.  It touches no
game arithmetic.
"""


def colored(text, color=None, on_color=None, attrs=None, **_kw):
    return text
