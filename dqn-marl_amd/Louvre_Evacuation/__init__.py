"""Drop-in mirror of the reference's Louvre_Evacuation package (envs / agents /
runners / utils) whose env step and DQN learner run on MI355X HIP kernels
(evacx, libevacx.so). Run from dqn-marl_amd/:  python -m Louvre_Evacuation.main --train_dqn
"""
import os as _os
import sys as _sys

_root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _root not in _sys.path:
    _sys.path.insert(0, _root)
