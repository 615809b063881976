"""Writes tests/golden/component_members.txt: every engine member the reference ROS component
reaches through `m_fusion->` (src/gpu_depthmap_fusion_component.cpp), one name per line with the
number of uses - the list tests/test_objects.py checks against include/gdf_fusion.hpp.  Run here,
where the reference checkout is (it is not on the GPU box; the list is committed):

    python tests/golden/make_component_members.py /root/reference
"""
import collections
import os
import re
import sys

src = open(os.path.join(sys.argv[1], "src", "gpu_depthmap_fusion_component.cpp")).read()
names = collections.Counter(re.findall(r"m_fusion->([A-Za-z_][A-Za-z_0-9]*)", src))
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "component_members.txt")
with open(out, "w") as f:
    for n in sorted(names):
        f.write(f"{n} {names[n]}\n")
print(out, len(names))
