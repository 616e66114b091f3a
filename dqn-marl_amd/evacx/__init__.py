"""evacx -- MI355X-native evacuation CA + DQN hot path (host side).

The compute path is the HIP library ``libevacx.so`` (dqn-marl_amd/csrc, C-ABI in
include/evacx.h); this package holds the host logic around it: the layout
table builder, the ctypes binding and the vectorised env / learner drivers.
"""
