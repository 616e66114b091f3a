"""CLI entry point: python -m Louvre_Evacuation.main --train_dqn (reference main.py:19-26)."""
import argparse
import os
import sys

_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _root not in sys.path:
    sys.path.insert(0, _root)

from Louvre_Evacuation.runners.train_dqn import main as train_dqn_main  # noqa: E402


def main():
    parser = argparse.ArgumentParser(description="Louvre Evacuation RL (MI355X)")
    parser.add_argument("--train_dqn", action="store_true", help="Train DQN agent")
    args = parser.parse_args()
    if args.train_dqn:
        train_dqn_main()
    else:
        print("specify an action, e.g. --train_dqn")


if __name__ == "__main__":
    main()
