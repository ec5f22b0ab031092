# Window simulation for the streamed maze RNG (apg_maze.hpp): per DFS iteration of a 127 x 127 maze, the PCG64
# outputs it consumes (maze_fifo_sim.trace); a lane holds a window of W outputs refilled to full every P
# iterations (the memory phase) and stalls an iteration whose draws do not fit in what is left.  Prints the
# outputs per maze (for the precomputed stream length) and the iterations a lane loses to stalls.
import os
import sys

import numpy as np

src = open(os.path.join(os.path.dirname(__file__), "maze_fifo_sim.py")).read().split("T=[trace")[0]
exec(src)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = [trace(i * 31 + 7) for i in range(n)]
tot = np.array([sum(p) for p in T])
print("outputs/maze mean %.1f std %.1f max %d iters %d" % (tot.mean(), tot.std(), tot.max(), len(T[0])))
for W in (32, 48, 64):
    for P in (8, 16):
        extra = []
        for p in T:
            avail, it, i = W, 0, 0
            while i < len(p):
                if it % P == 0:
                    avail = W
                if p[i] <= avail:
                    avail -= p[i]
                    i += 1
                it += 1
            extra.append(it - len(p))
        print("W %d P %d stall iterations per maze: mean %.1f max %d" % (W, P, np.mean(extra), max(extra)))
