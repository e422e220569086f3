"""PrimitiveLanguageTeacher's describe / instruct (teachers/primitive_language.py:9-90)
over batched transitions.

describe() maps each action the student took to a word by what the action did,
learning the student's action -> word map as it goes (one map shared by every
call) and drawing from the shared `config.random` where a step says nothing (no
move, no inventory change).  The only per-step facts it reads are the position
difference and whether the inventory changed; the kernels report exactly those
as transition codes (include/craft.h craft_transition / craft_step_ex):

    0..3  moved by the coord_change of DOWN / UP / LEFT / RIGHT
    4     did not move, inventory changed
    5     did not move, inventory unchanged

so a batch of envs is described from one int8 per env (`describe_codes`,
`describe_batch`) with the reference's word choices and random draws, in the
reference's order.  The map learning is inherently sequential and stays on the
host; once the map holds all six actions, a batch is a table lookup.
"""
import numpy as np

WORDS = ("down", "up", "left", "right", "use", "stop")      # action index order (craft.py:25-31)
_INFER_ORDER = ("up", "down", "left", "right", "use", "stop")  # primitive_language.py:49
_MOVE_WORD = {0: "down", 1: "up", 2: "left", 3: "right"}      # coord_change diffs, :77-84
USE_CODE, IDLE_CODE = 4, 5


def codes_from_states(prev_pos, next_pos, prev_inv, next_inv):
    """Transition codes from explicit state pairs (for CraftState objects)."""
    dx, dy = next_pos[0] - prev_pos[0], next_pos[1] - prev_pos[1]
    if (dx, dy) == (0, 0):
        return USE_CODE if (np.asarray(next_inv) != np.asarray(prev_inv)).any() else IDLE_CODE
    return {(0, -1): 0, (0, 1): 1, (-1, 0): 2, (1, 0): 3}[(dx, dy)]


class PrimitiveLanguageTeacher:
    """describe / instruct of teachers/primitive_language.py with the same state
    (`student_action_map`) and the same use of the shared RandomState."""

    def __init__(self, random):
        self.student_action_map = {}
        self.random = random
        self._lut = None

    # teachers/primitive_language.py:17-34
    def instruct(self, world, action_seq):
        out = []
        for a in action_seq:
            a = int(a)
            if not 0 <= a < len(WORDS):
                raise AssertionError("action == world.actions.STOP.index")
            out.append(WORDS[a])
        return out

    # teachers/primitive_language.py:36-90, from transition codes
    def describe_codes(self, action_seq, codes):
        description = []
        m = self.student_action_map
        n = len(action_seq)
        for i, (action, code) in enumerate(zip(action_seq, codes)):
            action, code = int(action), int(code)
            action_str = m.get(action)
            if action_str is None and len(m) == len(WORDS) - 1:        # infer the last action
                recognized = list(m.values())
                for w in _INFER_ORDER:
                    if w not in recognized:
                        m[action] = w
                        action_str = w
                        break
            if action_str is None:
                if code == USE_CODE:
                    m[action] = "use"
                    action_str = "use"
                elif code == IDLE_CODE:
                    candidates = ["down", "up", "left", "right", "use"]
                    if i + 1 == n:                                      # i + 1 == len(state_seq) - 1
                        candidates.append("stop")
                    action_str = self.random.choice(candidates)
                elif code in _MOVE_WORD:
                    m[action] = _MOVE_WORD[code]
                    action_str = m[action]
                else:
                    raise ValueError(f"no transition to describe (code {code})")
            assert action_str is not None
            description.append(str(action_str))
        self._lut = None
        return description

    def describe(self, world, action_seq, state_seq):
        """The reference's signature, over CraftState-like objects (pos, inventory)."""
        codes = [codes_from_states(state_seq[i].pos, state_seq[i + 1].pos, state_seq[i].inventory,
                                   state_seq[i + 1].inventory) for i in range(len(action_seq))]
        return self.describe_codes(action_seq, codes)

    def describe_batch(self, actions, codes):
        """One single-action describe() per env, envs in order, as
        trainers/interactive_primitive_language.py:58-68 calls it; entries whose
        code is -1 (no step) get None.  actions / codes: [B] host or device."""
        actions = np.asarray(actions.cpu() if hasattr(actions, "cpu") else actions).astype(np.int64)
        codes = np.asarray(codes.cpu() if hasattr(codes, "cpu") else codes).astype(np.int64)
        out = [None] * len(actions)
        idx = np.nonzero(codes >= 0)[0]
        k = 0
        while k < len(idx) and len(self.student_action_map) < len(WORDS):
            i = idx[k]
            out[i] = self.describe_codes([actions[i]], [codes[i]])[0]
            k += 1
        if k < len(idx):                          # the map is complete: a table lookup
            if self._lut is None:
                self._lut = np.array([self.student_action_map.get(a, "") for a in range(len(WORDS))],
                                     dtype=object)
            rest = idx[k:]
            words = self._lut[actions[rest]]
            for i, w in zip(rest, words):
                out[i] = w
        return out
