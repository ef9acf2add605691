#include "../fccf-pcr_amd/csrc/pool.h"
#include <cstdio>
#include <chrono>
#include <thread>
#include <set>
#include <mutex>
int main(int argc,char**argv){
  fccf::Pool pool(atoi(argv[1]));
  for(int rep=0;rep<5;++rep){
    std::mutex mu; std::set<std::thread::id> ids;
    auto t0=std::chrono::steady_clock::now();
    pool.parallel_for(86,[&](int i){ {std::lock_guard<std::mutex> g(mu); ids.insert(std::this_thread::get_id());} volatile double x=0; for(long k=0;k<atol(argv[2]);++k) x+=1e-9; });
    printf("rep %d: %.1f us, threads used %zu\n",rep,std::chrono::duration<double,std::micro>(std::chrono::steady_clock::now()-t0).count(),ids.size());
    std::this_thread::sleep_for(std::chrono::milliseconds(rep%2?0:2));
  }
}
