cd ${GRAFT_REPO_ROOT}
bash tools/ab_wall.sh "C2 C3" lib/libraytracer_hip.so lib/ab/libraytracer_hip_abl1.so lib/ab/libraytracer_hip_abl2.so lib/ab/libraytracer_hip_abl3.so
EXTRA="--strip spheres,planes,lights" bash tools/ab_wall.sh "C2" lib/libraytracer_hip.so
