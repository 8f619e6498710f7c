// CPU model of the BPE merge loop's candidate filter over config K5 (tools only).
//   python tools/sig_filter_words.py /tmp/k5w && g++ -O2 -o /tmp/sfs tools/sig_filter_sim.cpp && /tmp/sfs /tmp/k5w
// Replays the golden merges over the distinct words (HF's order, pair -> words index) and, every 75
// merges, counts the words whose 64-bit signature admits the merge's pair without holding it:
// round 5's form (two bits per symbol over 64) against round 6's (symbols in the low 32 bits,
// adjacent pairs in the high 32; csrc/bpe_common.h).  Prints "merge m true T fp_round5 fp_round6".
#include <cstdio>
#include <string>
#include <cstdint>
#include <vector>
#include <unordered_map>
#include <unordered_set>
#include <algorithm>
using namespace std;

static inline uint64_t sb(uint32_t x){ return (1ull<<(x&63))|(1ull<<(((x*0x9E3779B1u)>>26)&63)); }
static inline uint64_t ss(uint32_t x){ return (1ull<<(x&31))|(1ull<<((x*0x9E3779B1u)>>27)); }
static inline uint64_t sp(uint32_t a,uint32_t b){ uint32_t q=(a*0x9E3779B1u+b)*0x85EBCA6Bu; return (1ull<<(32+(q>>27)))|(1ull<<(32+((q>>22)&31u))); }
int main(int argc, char** argv){
  if(argc<2){fprintf(stderr,"usage: %s DIR\n",argv[0]);return 2;}
  const std::string dir=argv[1];
  FILE* f=fopen((dir+"/words.bin").c_str(),"rb"); fseek(f,0,SEEK_END); long n=ftell(f)/4; fseek(f,0,SEEK_SET);
  vector<int32_t> raw(n); fread(raw.data(),4,n,f); fclose(f);
  vector<vector<int>> W; vector<int> C;
  for(long i=0;i<n;){int c=raw[i],L=raw[i+1]; C.push_back(c); W.emplace_back(raw.begin()+i+2,raw.begin()+i+2+L); i+=2+L;}
  f=fopen((dir+"/merges.bin").c_str(),"rb"); vector<int32_t> mr(1724*3); fread(mr.data(),4,mr.size(),f); fclose(f);
  int M=1724; int V=2048;
  vector<long> lsz(V,0);
  // pair -> words index
  unordered_map<uint64_t, unordered_set<int>> where;
  auto key=[](int a,int b){return ((uint64_t)a<<32)|(uint32_t)b;};
  for(size_t w=0;w<W.size();++w){
    vector<int> u(W[w]); sort(u.begin(),u.end()); u.erase(unique(u.begin(),u.end()),u.end());
    for(int t:u) lsz[t]++;
    for(size_t i=0;i+1<W[w].size();++i) where[key(W[w][i],W[w][i+1])].insert(w);
  }
  vector<long> rew(M);
  for(int m=0;m<M;++m){
    int a=mr[3*m],b=mr[3*m+1],nid=mr[3*m+2];
    if(m%75==0 && m>0){ long f0=0,f1=0,tp=0; uint64_t n0=sb(a)|sb(b), n1=ss(a)|ss(b)|sp(a,b);
      for(auto&s:W){ bool h=false; for(size_t i=0;i+1<s.size();++i) if(s[i]==a&&s[i+1]==b) h=true; if(h){tp++;continue;}
        uint64_t g0=0,g1=0; for(size_t i=0;i<s.size();++i){ g0|=sb(s[i]); g1|=ss(s[i]); if(i) g1|=sp(s[i-1],s[i]); }
        f0+=((g0&n0)==n0); f1+=((g1&n1)==n1); }
      printf("merge %d true %ld %ld %ld\n",m,tp,f0,f1); fflush(stdout);}
    auto it=where.find(key(a,b)); long cntw=0;
    if(it!=where.end()){
      vector<int> ws(it->second.begin(),it->second.end());
      for(int w:ws){
        auto& s=W[w]; bool hit=false; vector<int> o;
        for(size_t i=0;i<s.size();){ if(i+1<s.size()&&s[i]==a&&s[i+1]==b){o.push_back(nid);i+=2;hit=true;} else o.push_back(s[i++]); }
        if(!hit) continue;
        cntw++;
        for(size_t i=0;i+1<o.size();++i) if(o[i]==nid||o[i+1]==nid) where[key(o[i],o[i+1])].insert(w);
        s=o;
      }
    }
    rew[m]=cntw; lsz[nid]=cntw;  // list of new token = words rewritten
  }
  // greedy passes
  vector<pair<int,int>> passes; // [start,end)
  int i=0; while(i<M){ int s=i; i++; 
    while(i<M && i-s<8){ int a=mr[3*i],b=mr[3*i+1]; bool ok=true;
      for(int k=s;k<i;++k){int ak=mr[3*k],bk=mr[3*k+1]; if(ak==bk||b==ak||a==bk) ok=false; }
      if(!ok) break; ++i; }
    passes.push_back({s,i}); }
  printf("passes %zu\n",passes.size());
  // need lsz at the time: base lsz initial; merged lsz set at creation (creation precedes use)
  long thr[]={20000,50000,100000,200000,400000};
  for(long T:thr){ int cnt=0; double tot=0; for(auto&p:passes){ long c=0; for(int m=p.first;m<p.second;++m){int a=mr[3*m],b=mr[3*m+1]; c+=min(lsz[a],lsz[b]);} if(c<=T){cnt++; tot+=c;} }
    printf("thr %ld: list passes %d, mean entries %.0f\n",T,cnt,cnt?tot/cnt:0); }
  // print sample
  for(size_t p=0;p<passes.size();p+=12){ long c=0,r=0; for(int m=passes[p].first;m<passes[p].second;++m){int a=mr[3*m],b=mr[3*m+1]; c+=min(lsz[a],lsz[b]); r+=rew[m];} printf("pass %zu merges %d list %ld rewritten %ld\n",p,passes[p].second-passes[p].first,c,r);}
}
