tools/ab_multi.sh "ab_base tree ab_min2 ab_min4" dragon && mv gpurun_out/par.log gpurun_out/par_tree.log && V=persist4 tools/ab_multi.sh "tree ab_p4tq" sportscar car_boxed
