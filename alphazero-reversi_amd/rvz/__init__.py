"""rvz — MI355X-native Reversi self-play engine (env + MCTS hot path of AlphaZero-Reversi).

Drop-in classes mirroring the reference's API (src/game, src/mcts, src/self_play):
    ReversiGame, Board      single-game rules, run in the HIP kernels
    MCTS                    search / get_action_probs / update_with_move
    SelfPlay                generate_games / generate_training_data, games in lockstep
Batched core:
    Engine                  n games + trees resident in HBM, C-ABI of include/rvz.h
    SelfPlayRunner          one ply per call, HIP-graph capturable
    LaneRunner              independent lanes of SelfPlayRunners, one stream each, one graph
    AlphaZeroNetwork, LeafEvaluator   the policy/value net at the evaluation boundary
"""
from ._lib import RvzError, load  # noqa: F401
from .engine import (Engine, board_apply, board_canonical, board_legal,  # noqa: F401
                     policy_softmax)
from .game import Board, ReversiGame  # noqa: F401
from .mcts import MCTS  # noqa: F401
from .network import (AlphaZeroNetwork, LeafEvaluator, ModuleEvaluator,  # noqa: F401
                      load_reference_state_dict)
from .selfplay import LaneRunner, SelfPlay, SelfPlayRunner  # noqa: F401

__version__ = "0.1.0"
