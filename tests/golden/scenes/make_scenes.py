"""Writes the .spray scene descriptions used by the tests and bench.

wavelets64.spray: 64 copies of wavelet.ply on a 4x4x4 translated grid, the
scene of the reference's examples/wavelets64 run (one point light at
(0, 500, 1000), diffuse white material, object bound [-10,-10,-10]-
[10,9.324713,10], translations x,z in {0,20,40,60}, y in steps of
19.324713; domain order x fastest, then y, then z).
wavelet2.spray: the two-domain example (wavelet0.ply / wavelet1.ply).
Run: python tests/golden/scenes/make_scenes.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def wavelets64():
    lines = ["# light <type> <position x y z> <intensity r g b> (point light)",
             "light point 0 500 1000 1 1 1", ""]
    dy = 19.324713
    k = 0
    for z in range(4):
        for y in range(4):
            for x in range(4):
                lines += ["# domain %d" % k, "domain", "file wavelet.ply",
                          "mtl diffuse 1 1 1",
                          "bound -10.000000 -10.000000 -10.000000 10.000000 9.324713 10.000000",
                          "face 5480", "vertex 2840",
                          "translate %.6f %.6f %.6f" % (20.0 * x, dy * y, 20.0 * z), ""]
                k += 1
    return "\n".join(lines)


def wavelet2():
    return "\n".join([
        "light point -20 20 20 .2 .2 .2", "light diffuse .1 .1 .1", "",
        "domain", "file wavelet1.ply", "vertex 958", "face 1748",
        "bound 0 -10 -10 6.612539768218994 10 10", "mtl diffuse 1 1 1", "",
        "domain", "file wavelet0.ply", "vertex 909", "face 1684",
        "bound -6.036099910736084 -10 -10 0 10 10", "mtl diffuse 1 1 1", ""])


def wavelet1():
    return "\n".join([
        "light point 0 500 1000 1 1 1", "",
        "domain", "file wavelet.ply", "mtl diffuse 1 1 1",
        "bound -10.000000 -10.000000 -10.000000 10.000000 9.324713 10.000000",
        "face 5480", "vertex 2840", ""])


if __name__ == "__main__":
    for name, body in [("wavelets64.spray", wavelets64()),
                       ("wavelet2.spray", wavelet2()),
                       ("wavelet1.spray", wavelet1())]:
        with open(os.path.join(HERE, name), "w") as f:
            f.write(body)
    print("ok")
