/* sync_sim.c -- CPU model of the entropy self-synchronisation (speculative warm-up + Jacobi sync
 * rounds) on one JPEG: prints the symbols/bits each phase decodes.  Design tool, not product.
 * build: gcc -O2 -w -o /tmp/sync_sim tools/sync_sim.c -lm ; run: /tmp/sync_sim img.jpg SUB_BITS WARM_BITS */
#include "../oracle/sdsj_oracle.c"  /* test infrastructure: the oracle's parser and tables */
#include <stdio.h>
static uint8_t *U; static size_t UN;
static int getb(uint64_t p, int n){ uint32_t v=0; for(int i=0;i<n;i++){uint64_t q=p+i; int bit = q/8<UN ? (U[q/8]>>(7-q%8))&1 : 0; v=(v<<1)|bit;} return v; }
static int hdec(uint64_t *p, const htable_t *t){ int l=1; int code=getb(*p,1); (*p)++; while(code>t->maxcode[l]){ code=(code<<1)|getb(*p,1); (*p)++; l++; if(l>16) return 0;} return t->vals[(code+t->valoffset[l])&0xFF]; }
int blkcomp[10], bpm;
static uint64_t dblock(uint64_t p, jpeg_t *j, int c){ comp_t *cp=&j->comp[c]; int s=hdec(&p,&j->dc[cp->td]); if(s>16) s=16; p+=s; for(int k=1;k<64;k++){int sym=hdec(&p,&j->ac[cp->ta]); int r=sym>>4; s=sym&15; if(s){k+=r; p+=s;} else { if(r!=15) break; k+=15;}} return p; }
#define MAXR 4096
typedef struct { uint64_t start,end; uint64_t rp[MAXR]; int rb[MAXR]; int nrec; uint64_t ep; int eph; uint64_t exit_p; int exit_ph; } sub_t;
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); static uint8_t d[1<<24]; size_t n=fread(d,1,sizeof d,f); fclose(f);
  jpeg_t j; memset(&j,0,sizeof j); if(parse_headers(d,n,&j)||setup_geometry(&j)){printf("parse fail\n");return 1;}
  U=malloc(n); UN=0; for(size_t i=j.entropy_off;i<n;i++){ if(d[i]==0xFF){ if(d[i+1]==0){U[UN++]=0xFF;i++;continue;} else break;} U[UN++]=d[i]; }
  bpm=0; for(int c=0;c<j.ncomp;c++) for(int k=0;k<j.comp[c].h*j.comp[c].v;k++) blkcomp[bpm++]=c;
  uint64_t total_bits = UN*8;
  int SB = atoi(argv[2]); int W = argc>3?atoi(argv[3]):0; int kRec = argc>4?atoi(argv[4]):64;
  int ns = (total_bits+SB-1)/SB; sub_t *S = calloc(ns,sizeof(sub_t));
  long long specbits=0, syncbits=0;
  for(int i=0;i<ns;i++){ S[i].start=(uint64_t)i*SB; S[i].end=S[i].start+SB; if(S[i].end>total_bits) S[i].end=total_bits;
    // warmup: decode from start-W (phase 0) until >= start
    uint64_t q = i? (S[i].start>W? S[i].start-W:0) : 0; int ph=0;
    if(i){ while(q<S[i].start){ q=dblock(q,&j,blkcomp[ph]); ph=(ph+1)%bpm; } } 
    specbits += q - (i?(S[i].start>W?S[i].start-W:0):0);
    S[i].ep=q; S[i].eph=ph; uint64_t q0=q;
    int nr=0; while(q<S[i].end){ q=dblock(q,&j,blkcomp[ph]); if(nr<kRec){S[i].rp[nr]=q; S[i].rb[nr]=ph;} nr++; ph=(ph+1)%bpm; }
    S[i].nrec = nr<kRec?nr:kRec; S[i].exit_p=q; S[i].exit_ph=ph; specbits += q-q0; }
  int rounds=0; int ntasks_tot=0; long long crit=0;
  for(;;){ int nt=0; uint64_t nep[ns]; int neph[ns]; int need[ns];
    for(int i=0;i<ns;i++){ need[i]=0; if(i && (S[i-1].exit_p!=S[i].ep || S[i-1].exit_ph!=S[i].eph)){ need[i]=1; nep[i]=S[i-1].exit_p; neph[i]=S[i-1].exit_ph; nt++; } }
    if(!nt) break; rounds++; ntasks_tot+=nt; uint64_t mx=0;
    uint64_t nx[ns]; int nxph[ns];
    for(int i=0;i<ns;i++) if(need[i]){ uint64_t q=nep[i]; int ph=neph[i]; int ri=0; int merged=0; uint64_t q0=q;
        while(q<S[i].end){ int bph=ph; q=dblock(q,&j,blkcomp[ph]); ph=(ph+1)%bpm; while(ri<S[i].nrec && S[i].rp[ri]<q) ri++; if(ri<S[i].nrec && S[i].rp[ri]==q && S[i].rb[ri]==bph){merged=1;break;} }
        syncbits += q-q0; if(q-q0>mx) mx=q-q0; if(merged){ nx[i]=S[i].exit_p; nxph[i]=S[i].exit_ph; } else { nx[i]=q; nxph[i]=ph; } }
    crit+=mx;
    for(int i=0;i<ns;i++) if(need[i]){ S[i].ep=nep[i]; S[i].eph=neph[i]; S[i].exit_p=nx[i]; S[i].exit_ph=nxph[i]; }
  }
  printf("tasks=%d crit=%lld ",ntasks_tot,crit); printf("SB=%d W=%d nsub=%d rounds=%d spec=%.2fx sync=%.2fx of %llu bits\n",SB,W,ns,rounds,(double)specbits/total_bits,(double)syncbits/total_bits,(unsigned long long)total_bits);
}
