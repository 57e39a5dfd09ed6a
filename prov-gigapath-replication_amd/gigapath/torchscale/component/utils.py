"""Small helpers of the reference's component/utils.py that the slide-encoder path uses."""


def padding_to_multiple_of(n: int, mult: int) -> int:
    """Elements to add so that n becomes a multiple of mult (component/utils.py:7-11)."""
    return (-n) % mult
