"""Extrude a 2D gmsh 2.2 quad mesh into a 3D hex mesh (gmsh 2.2): layers along z, boundary lines
become boundary quads with the same physical tag, the z = 0 / z = Lz faces get tags `--ztags`.
Used to author the 3D flow-past-a-cylinder case of BASELINE configs[4] from the reference's 2D
examples/03-cylinder mesh (tests/golden/meshes/cylinder_structured.msh).
Usage: python tools/extrude_gmsh.py in.msh out.msh --layers 4 --length 2 --ztags 4 5"""
import argparse


def read22(path):
    L = open(path).read().split("\n")
    i = L.index("$Nodes")
    n = int(L[i + 1])
    nodes = {}
    for l in L[i + 2:i + 2 + n]:
        t = l.split()
        nodes[int(t[0])] = tuple(float(v) for v in t[1:4])
    i = L.index("$Elements")
    m = int(L[i + 1])
    elems = []
    for l in L[i + 2:i + 2 + m]:
        t = [int(v) for v in l.split()]
        typ, ntag = t[1], t[2]
        elems.append((typ, t[3:3 + ntag], t[3 + ntag:]))
    return nodes, elems


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("inp")
    ap.add_argument("out")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--length", type=float, default=2.0)
    ap.add_argument("--ztags", type=int, nargs=2, default=(4, 5))
    a = ap.parse_args()
    nodes, elems = read22(a.inp)
    ids = sorted(nodes)
    nn = len(ids)
    idx = {g: k for k, g in enumerate(ids)}
    nid = lambda g, j: j * nn + idx[g] + 1  # 1-based node tag of 2D node g in layer j
    out_nodes = []
    for j in range(a.layers + 1):
        z = a.length * j / a.layers
        for g in ids:
            x, y, _ = nodes[g]
            out_nodes.append((nid(g, j), x, y, z))
    out_el = []
    for typ, tags, vs in elems:
        phys = tags[0]
        for j in range(a.layers):
            if typ == 3:  # quad -> hex (bottom face then top face, same rotation)
                out_el.append((5, phys, [nid(v, j) for v in vs] + [nid(v, j + 1) for v in vs]))
            elif typ == 1:  # boundary line -> boundary quad
                p, q = vs
                out_el.append((3, phys, [nid(p, j), nid(q, j), nid(q, j + 1), nid(p, j + 1)]))
        if typ == 3:
            out_el.append((3, a.ztags[0], [nid(v, 0) for v in vs]))
            out_el.append((3, a.ztags[1], [nid(v, a.layers) for v in vs]))
    with open(a.out, "w") as f:
        f.write("$MeshFormat\n2.2 0 8\n$EndMeshFormat\n$Nodes\n%d\n" % len(out_nodes))
        for t, x, y, z in out_nodes:
            f.write("%d %.12g %.12g %.12g\n" % (t, x, y, z))
        f.write("$EndNodes\n$Elements\n%d\n" % len(out_el))
        for k, (typ, phys, vs) in enumerate(out_el, 1):
            f.write("%d %d 2 %d %d %s\n" % (k, typ, phys, phys, " ".join(map(str, vs))))
        f.write("$EndElements\n")


if __name__ == "__main__":
    main()
