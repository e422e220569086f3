"""Host logic of psketch_amd.rollout that runs without a GPU: the graph cache's key on the
student's act (a bound method is a new object on every attribute access, so identity would
re-capture every rollout; the cache holds it weakly so it does not keep the model alive)."""
import gc

from psketch_amd import rollout as R


class Student:
    def __init__(self):
        self.calls = 0

    def act(self, obs, t):
        self.calls += 1
        return obs


def test_bound_method_matches_across_accesses():
    s = Student()
    ref = R._weak_act(s.act)
    assert s.act is not s.act                       # why identity was the wrong test
    assert R._same_act(ref, s.act)
    assert not R._same_act(ref, Student().act)      # same function, another object


def test_cache_does_not_keep_the_student_alive():
    s = Student()
    ref = R._weak_act(s.act)
    del s
    gc.collect()
    assert ref() is None
    assert not R._same_act(ref, Student().act)


def test_plain_functions_and_closures():
    def f(obs, t):
        return obs
    ref = R._weak_act(f)
    assert R._same_act(ref, f)
    assert not R._same_act(ref, lambda obs, t: obs)
    ref_builtin = R._weak_act(len)                  # no weak references: held strongly
    assert R._same_act(ref_builtin, len)
