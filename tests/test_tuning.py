"""CPU checks of the autotuner policy and the attribution knobs' parsing (ops/tuning.py,
ops/conv_hip.py): without a GPU the tuner never times anything, returns the default and caches
it; the weight-gradient candidate whitelist parses ranges and lists."""
from simclr_amd.ops import conv_hip, tuning


def test_pick_without_gpu_returns_default_and_caches():
    calls = []
    key = ("test-tuning-default",)
    tuning._CACHE.pop(key, None)
    v = tuning.pick(key, [2, 4, 6], 4, lambda c: calls.append(c))
    assert v == 4 and calls == []
    assert tuning.cached(key) == 4
    # a cached key returns before the candidate list is even looked at
    assert tuning.pick(key, [], 9, lambda c: calls.append(c)) == 4
    tuning._CACHE.pop(key, None)


def test_pick_default_outside_candidates_falls_back_to_first():
    key = ("test-tuning-first",)
    tuning._CACHE.pop(key, None)
    assert tuning.pick(key, [3, 5], 7, lambda c: None) == 3
    tuning._CACHE.pop(key, None)


def test_rounds_default():
    assert tuning.ROUNDS >= 1
