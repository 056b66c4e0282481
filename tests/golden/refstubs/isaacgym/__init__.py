"""Name-only stand-in for the absent Isaac Gym package (fixture generation only).

Used exclusively by tests/golden/make_golden.py to import the reference's own
Python in this container.  Nothing here simulates physics: the fake gym object
in tests/golden/make_golden.py writes the post-physics state chosen by the
harness into the tensors the reference reads.
"""
